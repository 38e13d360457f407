#!/bin/bash
# Round-4 session I: the D = 1 kernel inverse FFTs in pairs / fours vs one at a time (A/B)
# variants) A/B, interleaved and bit-compared. -> gpurun_out/r04i/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04i
mkdir -p "$OUT"
timeout -k 10 300 tools/exp/_build_fft_ab/fft_bench > "$OUT/d1np_ab.log" 2>&1
rc=$?; echo "d1np ab rc=$rc"; cat "$OUT/d1np_ab.log"; exit $rc
