#!/bin/bash
# Round-4 session F: intra-workgroup block scheduling (LDS counter) vs static rounds - stamps with raw
# dumps and an interleaved A/B; the FFT parity tests on the product build; the WS abort diagnostic
# (resident-API-conforming sequence). -> gpurun_out/r04f/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04f
mkdir -p "$OUT"
FFT_BENCH_STAMPS=1 FFT_BENCH_STAMP_DUMP=$OUT/st timeout -k 10 200 tools/exp/_build_fft/fft_bench > "$OUT/stamps.log" 2>&1
rc=$?; echo "stamps rc=$rc"; cat "$OUT/stamps.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tools/exp/_build_fft_ab/fft_bench > "$OUT/sched_ab.log" 2>&1
rc=$?; echo "sched ab rc=$rc"; cat "$OUT/sched_ab.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_fft_fir.py > "$OUT/fft_tests.log" 2>&1
rc=$?; echo "fft tests rc=$rc"; tail -3 "$OUT/fft_tests.log"; [ $rc -eq 0 ] || exit $rc
GSDR_LIB=$PWD/cuda-sdr_amd/lib_diag/libgpusdrpipeline.so timeout -k 10 180 python3 -u tools/exp/ws_abort_diag.py > "$OUT/ws_abort_diag.log" 2>&1
rc=$?; echo "ws diag rc=$rc"; grep -v amdgpu.ids "$OUT/ws_abort_diag.log" | head -20; exit $rc
