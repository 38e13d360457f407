#!/bin/bash
# Board power / GFX clock while one FFT variant loops (tools/exp/run_fft_variants.sh build first).
# Usage (GPU box): bash tools/exp/fft_power_probe.sh <variant> [reps]
cd "$(dirname "$0")/../.."
V=${1:-base}
( for i in $(seq 1 16); do amd-smi metric -p -c -g 0 2>&1 | grep -E "SOCKET_POWER|GFX_0|CLK:" | head -4; echo ---; sleep 0.5; done ) > gpurun_out/power_$V.log &
P=$!
FFT_BENCH_LOOP=$V FFT_BENCH_REPS=${2:-16000} timeout -k 10 120 tools/exp/_build_fft/fft_bench > gpurun_out/power_bench_$V.log 2>&1
wait $P
