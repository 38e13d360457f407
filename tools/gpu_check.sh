#!/bin/bash
# GPU-box check after a kernel change: the full -m gpu suite, then the bench on the C3 and C5
# workloads (no CPU baseline). Each step has its own time limit; a crash or timeout ends the run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
        echo "== $name rc=$rc"; tail -n 4 "$OUT/$name.log" | cut -c1-900
        if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL $name"; exit $rc; fi; }
run pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
run bench_c3 300 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline
run bench_c5 300 python bench.py --workload c5 --steps 10 --warmup 3 --no-cpu-baseline
