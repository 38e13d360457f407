#!/bin/bash
# A/B and diagnostic builds of libgpusdrpipeline.so, out of the product tree's way:
#   tools/build_variant.sh NAME [EXTRA_FLAGS...]
# builds tools/exp/_ablib/NAME/libgpusdrpipeline.so (objects in tools/exp/_ablib/NAME/build) with the
# given -D switches; load it with GSDR_LIB=<that path>. Its gsdrAmdBuildId folds EXTRA_FLAGS in, so
# test_library_matches_source_tree rejects it as the product library. Variants used in the record:
#   noz   -DGSDR_WS_RING_ZERO=0  the r04 stale-LDS defect (test_fused_chain_ignores_stale_lds must fail)
#   diag  -DGSDR_WS_DIAG=1       bounds counters of the fused audio stage (tools/exp/ws_abort_diag.py)
#   waits -DGSDR_WS_WAITS=1      hand-off wait profile (tools/exp/c5_waits_probe.py)
set -euo pipefail
name=$1
shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/tools/exp/_ablib/$name
mkdir -p "$out"
make -s -j"${JOBS:-8}" -C "$root/cuda-sdr_amd" BUILD="$out/build" LIBDIR="$out" EXTRA_FLAGS="$*"
echo "$out/libgpusdrpipeline.so"
