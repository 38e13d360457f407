#!/bin/bash
# Build and time variants of csrc/kernels/fir_cf_mfma.hip (same scheme as run_i8_variants.sh).
set -eu
cd "$(dirname "$0")/../.."
OUT=tools/exp/_build_cf
KSRC=cuda-sdr_amd/csrc/kernels/fir_cf_mfma.hip
# the attribution switches live in a patch, applied to a copy (the shipped kernel has none)
ASRC=${OUT:-tools/exp}/fir_cf_mfma_attr.hip
VARIANTS=${VARIANTS:-"base|
nosplit|-DGSDR_CF_EXPERIMENT=1
nomfma|-DGSDR_CF_EXPERIMENT=2
noload|-DGSDR_CF_EXPERIMENT=4
noreduce|-DGSDR_CF_EXPERIMENT=8
nostats|-DGSDR_CF_EXPERIMENT=16
mfma_only|-DGSDR_CF_EXPERIMENT=29
no_mfma_no_split|-DGSDR_CF_EXPERIMENT=3"}
if [ "${1:-build}" = build ]; then
  mkdir -p $OUT
  patch -s -o $ASRC $KSRC tools/exp/attribution/fir_cf_mfma.patch || echo "attribution patch does not apply to the current kernel (variants naming a source still build)"
  decls=""; table=""; objs=""; i=0
  while IFS='|' read -r name flags; do
    [ -z "$name" ] && continue
    hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Iinclude -Icuda-sdr_amd/csrc/kernels -mllvm -amdgpu-mfma-vgpr-form \
      -Dgsdr_amd=c$i $flags -c $ASRC -o $OUT/c$i.o &
    decls="$decls DECL($i)"; table="$table {\"$name\", c$i::launchFirCfMfma, c$i::wsReadStamps},"; objs="$objs $OUT/c$i.o"
    i=$((i+1))
  done <<< "$VARIANTS"
  wait
  sed "s/namespace v##N/namespace c##N/" tools/exp/cf_bench.cpp > $OUT/cf_bench.cpp
  hipcc --offload-arch=gfx950 -O2 -std=c++20 "-DVARIANT_DECLS=$decls" "-DVARIANT_TABLE=$table" -c $OUT/cf_bench.cpp -o $OUT/main.o
  hipcc --offload-arch=gfx950 $OUT/main.o $objs -o $OUT/cf_bench
  echo built $OUT/cf_bench
else
  timeout -k 10 300 $OUT/cf_bench
fi
