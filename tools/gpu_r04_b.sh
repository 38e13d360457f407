#!/bin/bash
# Round-4 session B: the FFT kernel's in-kernel clock (wave stamps after 2.5 s of back-to-back
# launches, per attribution variant; tools/exp/run_fft_variants.sh with STAMPS=1). -> gpurun_out/r04b/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04b
mkdir -p "$OUT"
FFT_BENCH_STAMPS=1 timeout -k 10 300 tools/exp/_build_fft/fft_bench > "$OUT/stamps.log" 2>&1
rc=$?; echo "stamps rc=$rc"; cat "$OUT/stamps.log"; exit $rc
