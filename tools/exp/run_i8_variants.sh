#!/bin/bash
# Build and time variants of csrc/kernels/fir_i8_mfma.hip: each line of VARIANTS is
# "name|extra flags[|source file]"; every variant is compiled into its own namespace (-Dgsdr_amd=vN).
# Usage: bash tools/exp/run_i8_variants.sh build   (here, cross-compile)
#        bash tools/exp/run_i8_variants.sh run     (GPU box)
set -eu
cd "$(dirname "$0")/../.."
OUT=tools/exp/_build
KSRC=cuda-sdr_amd/csrc/kernels/fir_i8_mfma.hip
# the attribution switches live in a patch, applied to a copy (the shipped kernel has none)
ASRC=${OUT:-tools/exp}/fir_i8_mfma_attr.hip
VARIANTS=${VARIANTS:-"base|
base_clk|-DGSDR_I8_EXPERIMENT=32
bpc2|-DGSDR_I8_BLOCKS_PER_CU=2
tiles1|-DGSDR_I8_TILES_PER_WAVE=1
tiles1_clk|-DGSDR_I8_TILES_PER_WAVE=1 -DGSDR_I8_EXPERIMENT=32"}
if [ "${1:-build}" = build ]; then
  mkdir -p $OUT
  patch -s -o $ASRC $KSRC tools/exp/attribution/fir_i8_mfma.patch || echo "attribution patch does not apply to the current kernel (variants naming a source still build)"
  decls=""; table=""; objs=""; i=0
  while IFS='|' read -r name flags src; do
    [ -z "$name" ] && continue
    hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Iinclude -Icuda-sdr_amd/csrc/kernels -mllvm -amdgpu-mfma-vgpr-form \
      -Dgsdr_amd=v$i $flags -c ${src:-$ASRC} -o $OUT/v$i.o &
    decls="$decls DECL($i)"; table="$table {\"$name\", v$i::launchFirI8Mfma},"; objs="$objs $OUT/v$i.o"
    i=$((i+1))
  done <<< "$VARIANTS"
  wait
  hipcc --offload-arch=gfx950 -O2 -std=c++20 "-DVARIANT_DECLS=$decls" "-DVARIANT_TABLE=$table" \
    -c tools/exp/i8_bench.cpp -o $OUT/main.o
  hipcc --offload-arch=gfx950 $OUT/main.o $objs -o $OUT/i8_bench
  echo built $OUT/i8_bench
else
  timeout -k 10 300 $OUT/i8_bench
fi
