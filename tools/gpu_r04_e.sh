#!/bin/bash
# Round-4 session E: FFT kernel wave stamps with raw dumps (base vs tail-balancing pool), the pool
# round-count A/B (interleaved, bit-compared), the phase-pair kernel at R = 2 / 256 threads, the WS
# abort diagnostic. -> gpurun_out/r04e/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04e
mkdir -p "$OUT"
FFT_BENCH_STAMPS=1 FFT_BENCH_STAMP_DUMP=$OUT/st timeout -k 10 200 tools/exp/_build_fft/fft_bench > "$OUT/stamps.log" 2>&1
rc=$?; echo "stamps rc=$rc"; cat "$OUT/stamps.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/exp/_build_fft_ab/fft_bench > "$OUT/pool_ab.log" 2>&1
rc=$?; echo "pool ab rc=$rc"; cat "$OUT/pool_ab.log"; [ $rc -eq 0 ] || exit $rc
PT="python -u -m pytest -x -v --timeout 180 --timeout-method thread"
GSDR_LIB=$PWD/cuda-sdr_amd/lib_dec/libgpusdrpipeline.so timeout -k 10 300 $PT tests/test_gpu_parity.py -k "phase_pair" > "$OUT/dec_r2_t256.log" 2>&1
rc=$?; echo "dec R2 T256 rc=$rc"; tail -3 "$OUT/dec_r2_t256.log"; [ $rc -eq 0 ] || exit $rc
GSDR_LIB=$PWD/cuda-sdr_amd/lib_diag/libgpusdrpipeline.so timeout -k 10 180 python3 -u tools/exp/ws_abort_diag.py > "$OUT/ws_abort_diag.log" 2>&1
rc=$?; echo "ws diag rc=$rc"; grep -v amdgpu.ids "$OUT/ws_abort_diag.log"; exit $rc
