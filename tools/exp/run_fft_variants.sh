#!/bin/bash
# Build (here) and run (on the GPU box) attribution variants of csrc/kernels/fir_fft.hip.
#   bash tools/exp/run_fft_variants.sh build   # CPU container
#   bash tools/exp/run_fft_variants.sh run     # GPU box
# GSDR_FFT_EXP bits (in the kernel source, 0 in the product build): 1 no FFT math, 2 no global
# loads, 4 no LDS transposition, 8 no guard, 16 no stores. STAMPS=1 builds every variant with the
# in-kernel clock stamps (GSDR_FFT_STAMPS; run with FFT_BENCH_STAMPS=1). An optional third field
# names another source file (e.g. a saved baseline).
set -eu
cd "$(dirname "$0")/../.."
OUT=${OUT:-tools/exp/_build_fft}
KSRC=cuda-sdr_amd/csrc/kernels/fir_fft.hip
VARIANTS=${VARIANTS:-"base|
nofft|-DGSDR_FFT_EXP=1
noload|-DGSDR_FFT_EXP=2
notrans|-DGSDR_FFT_EXP=4
noguard|-DGSDR_FFT_EXP=8
nostore|-DGSDR_FFT_EXP=16
fft_only|-DGSDR_FFT_EXP=30
load_only|-DGSDR_FFT_EXP=29"}
STAMPFLAG=""
[ "${STAMPS:-0}" = 1 ] && STAMPFLAG="-DGSDR_FFT_STAMPS=1"
if [ "${1:-build}" = build ]; then
  mkdir -p $OUT
  decls=""; table=""; objs=""; i=0
  while IFS='|' read -r name flags src; do
    [ -z "$name" ] && continue
    hipcc --offload-arch=gfx950 -O3 -std=c++20 -fPIC -Iinclude -Icuda-sdr_amd/csrc/kernels \
      -Dgsdr_amd=f$i -DgsdrAmdSetFftGuard=f${i}_sg -DgsdrAmdGetFftGuard=f${i}_gg -DgsdrAmdFftDirectBlocks=f${i}_db \
      $STAMPFLAG $flags -c ${src:-$KSRC} -o $OUT/f$i.o &
    decls="$decls DECL($i)"; table="$table {\"$name\", f$i::launchPlain, f$i::fftStampsRead},"; objs="$objs $OUT/f$i.o"
    i=$((i+1))
  done <<< "$VARIANTS"
  wait
  hipcc --offload-arch=gfx950 -O2 -std=c++20 "-DVARIANT_DECLS=$decls" "-DVARIANT_TABLE=$table" -c tools/exp/fft_bench.cpp -o $OUT/main.o
  hipcc --offload-arch=gfx950 $OUT/main.o $objs -o $OUT/fft_bench
  echo built $OUT/fft_bench
else
  timeout -k 10 300 $OUT/fft_bench
fi
