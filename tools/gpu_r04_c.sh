#!/bin/bash
# Round-4 session C: FFT clock stamps; the native shard executor over RCCL (ring of one) and with an
# enqueue-only exchange; the phase-pair kernel at its other accepted block shape (R = 2, 256 threads)
# through its parity tests; the build-id check. -> gpurun_out/r04c/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04c
mkdir -p "$OUT"
FFT_BENCH_STAMPS=1 timeout -k 10 300 tools/exp/_build_fft/fft_bench > "$OUT/stamps.log" 2>&1
rc=$?; echo "stamps rc=$rc"; cat "$OUT/stamps.log"; [ $rc -eq 0 ] || exit $rc
PT="python -u -m pytest -x -v --timeout 180 --timeout-method thread"
timeout -k 10 600 $PT tests/test_shard_native_gpu.py tests/test_abi_exports.py tests/test_fft_fir.py -k "native_shard or library or exported or full_c4 or complex_taps"  > "$OUT/native_shard.log" 2>&1
rc=$?; echo "native shard rc=$rc"; tail -15 "$OUT/native_shard.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 $PT tests/test_filter_graph.py > "$OUT/filter_graph.log" 2>&1
rc=$?; echo "filter graph rc=$rc"; tail -3 "$OUT/filter_graph.log"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/exp/host_step_probe.py > "$OUT/host_step.log" 2>&1
rc=$?; echo "host step rc=$rc"; cat "$OUT/host_step.log"; [ $rc -eq 0 ] || exit $rc
GSDR_LIB=$PWD/cuda-sdr_amd/lib_dec/libgpusdrpipeline.so timeout -k 10 300 $PT tests/test_gpu_parity.py -k "phase_pair" > "$OUT/dec_r2_t256.log" 2>&1
rc=$?; echo "dec R2 T256 rc=$rc"; tail -5 "$OUT/dec_r2_t256.log"; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_r04_d.sh
