#!/bin/bash
# C5 (full AM chain executor) on the GPU box: bench lines (resident and chunked) + rocprofv3 trace.
set -e
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/c5.log 2>&1
timeout -k 10 300 python bench.py --workload c5 --c5-mode chunked --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/c5_chunked.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5 -o c5 -- python bench.py --workload c5 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/c5prof.log 2>&1
