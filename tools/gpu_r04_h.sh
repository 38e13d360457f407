#!/bin/bash
# Round-4 session H: XCD-contiguous workgroup order for the D >= 2 FFT kernel (+ non-temporal group
# variants) A/B, interleaved and bit-compared. -> gpurun_out/r04h/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04h
mkdir -p "$OUT"
timeout -k 10 300 tools/exp/_build_fft_ab/fft_bench > "$OUT/xcd_ab.log" 2>&1
rc=$?; echo "xcd ab rc=$rc"; cat "$OUT/xcd_ab.log"; exit $rc
