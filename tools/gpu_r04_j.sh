#!/bin/bash
# Round-4 session J: exchangeA in registers vs LDS (A/B + clock stamps)
# variants) A/B, interleaved and bit-compared. -> gpurun_out/r04j/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04j
mkdir -p "$OUT"
timeout -k 10 300 tools/exp/_build_fft_ab/fft_bench > "$OUT/xareg_ab.log" 2>&1
rc=$?; echo "xareg ab rc=$rc"; cat "$OUT/xareg_ab.log"; [ $rc -eq 0 ] || exit $rc
FFT_BENCH_STAMPS=1 timeout -k 10 200 tools/exp/_build_fft/fft_bench > "$OUT/stamps.log" 2>&1
rc=$?; echo "stamps rc=$rc"; cat "$OUT/stamps.log"; exit $rc
