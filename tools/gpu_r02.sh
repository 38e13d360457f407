#!/bin/bash
# Round-2 GPU check: sharded-path tests, the FFT tests, then the bench lines (C3 default, C2, C5
# sharded) and the multi-rank path on one GPU (gloo, ranks sharing cuda:0). Each step has its own
# time limit; a crash, abort or timeout ends the run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
        echo "== $name rc=$rc"; tail -n ${TAILN:-3} "$OUT/$name.log" | cut -c1-2500
        if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL $name"; exit $rc; fi; }
TAILN=15 run pytest_shard 300 python -u -m pytest tests/test_shard_gpu.py tests/test_fft_fir.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
run bench_c3 200 python bench.py --workload c3 --steps 20 --warmup 3 --no-cpu-baseline
run bench_c2 200 python bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline
run bench_c5 200 python bench.py --workload c5 --steps 20 --warmup 3 --no-cpu-baseline
run bench_c3_g2 200 python bench.py --workload c3 --gpus 2 --share-gpu --backend gloo --steps 10 --warmup 2
run bench_c5_g2 200 python bench.py --workload c5 --gpus 2 --share-gpu --backend gloo --steps 10 --warmup 2
