#!/bin/bash
# Build and time variants of csrc/kernels/fir_i8_ws4.hip at the fused C5 shape: each line of VARIANTS is
# "name|extra flags[|source file]" (default: the product source); every variant is compiled into its own namespace (-Dgsdr_amd=vN) with only the
# C5 instantiation (-DGSDR_W4_HARNESS). Usage: bash tools/exp/run_w4_variants.sh build   (here)
#                                             bash tools/exp/run_w4_variants.sh run     (GPU box)
set -eu
cd "$(dirname "$0")/../.."
OUT=tools/exp/_build_w4
VARIANTS=${VARIANTS:-"base|"}
if [ "${1:-build}" = build ]; then
  mkdir -p $OUT
  decls=""; table=""; objs=""; i=0
  while IFS='|' read -r name flags src; do
    [ -z "$name" ] && continue
    wflags=""; wfn=nullptr
    case "$flags" in *GSDR_WS_WAITS=1*) wflags="-DGSDR_W4_HARNESS_WAITS=w4w$i"; wfn=w4w$i; decls="$decls DECLW($i)";; esac
    sfn=nullptr
    case "$flags" in *GSDR_W4_STAMPS*) wflags="$wflags -DGSDR_W4_HARNESS_STAMPS=w4s$i"; sfn=w4s$i; decls="$decls DECLS($i)";; esac
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Iinclude -Icuda-sdr_amd/csrc/kernels \
      -mllvm -amdgpu-mfma-vgpr-form -Dgsdr_amd=v$i -DGSDR_W4_HARNESS=w4v$i $wflags $flags \
      -c ${src:-cuda-sdr_amd/csrc/kernels/fir_i8_ws4.hip} -o $OUT/v$i.o &
    decls="$decls DECL($i)"; table="$table {\"$name\", w4v$i, $wfn, $sfn},"; objs="$objs $OUT/v$i.o"
    i=$((i+1))
  done <<< "$VARIANTS"
  wait
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 -std=c++20 -Iinclude -Icuda-sdr_amd/csrc/kernels \
    "-DVARIANT_DECLS=$decls" "-DVARIANT_TABLE=$table" -c tools/exp/w4_bench.cpp -o $OUT/main.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 $OUT/main.o $objs -o $OUT/w4_bench
  echo built $OUT/w4_bench
else
  timeout -k 10 300 $OUT/w4_bench
fi
