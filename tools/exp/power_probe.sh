#!/bin/bash
# Sample board power / clocks while a variant loops (tools/exp/run_i8_variants.sh build first).
# Usage (GPU box): bash tools/exp/power_probe.sh <reps>
cd "$(dirname "$0")/../.."
( for i in $(seq 1 12); do amd-smi metric -p -c -g 0 2>&1 | grep -E "SOCKET_POWER|GFX_0|CLK|POWER" | head -8; echo ---; sleep 0.25; done ) > gpurun_out/power.log &
P=$!
REPS=${1:-60000} timeout -k 10 120 tools/exp/_build/i8_bench > gpurun_out/power_bench.log 2>&1
wait $P
