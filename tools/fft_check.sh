#!/bin/bash
# GPU-box iteration on the FFT FIR: its parity tests, then the C3 bench and a rocprofv3 kernel
# trace of it. Each step has its own limit; a crash/abort/timeout ends the run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
        echo "== $name rc=$rc"; tail -n ${TAILN:-6} "$OUT/$name.log" | cut -c1-1500
        if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL $name"; exit $rc; fi; }
TAILN=25 run pytest_fft 400 python -u -m pytest tests/test_fft_fir.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
run bench_c3 200 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline
run rocprof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c3" -o run -- python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline
find $OUT/prof_c3 -name "*kernel_stats.csv" -exec head -5 {} \;
