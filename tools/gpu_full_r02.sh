#!/bin/bash
# Round-2 full GPU validation: the whole -m gpu suite (one process), smoke(), the default bench
# (C3, with the CPU baseline) and the C2 / C5 lines. Each step has its own time limit; a crash,
# abort or timeout ends the run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/full; mkdir -p $OUT
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
        echo "== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log" | cut -c1-1500
        if [ $rc -ne 0 ]; then echo "FATAL $name"; exit $rc; fi; }
TAILN=6 run pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_default 400 python bench.py
run bench_c2 200 python bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline
run bench_c4 200 python bench.py --workload c4 --steps 20 --warmup 3 --no-cpu-baseline
run bench_c5 200 python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline
echo "full validation done"
