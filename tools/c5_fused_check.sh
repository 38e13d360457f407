#!/bin/bash
# GPU check of the fused C5 chain: the chain / shard / fused tests, then the C5 bench in its three modes.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/c5f
timeout -k 10 400 python -u -m pytest tests/test_am_fused.py tests/test_am_chain.py tests/test_shard_gpu.py tests/test_components_gpu.py \
  -m gpu -v --timeout 200 --timeout-method thread > gpurun_out/c5f/tests.log 2>&1
rc=$?
grep -E "FAILED|ERROR" gpurun_out/c5f/tests.log | head -20; tail -2 gpurun_out/c5f/tests.log
if [ $rc -ne 0 ]; then exit $rc; fi
for m in sharded resident chunked; do
  timeout -k 10 200 python -u bench.py --workload c5 --c5-mode $m --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/c5f/bench_$m.json 2> gpurun_out/c5f/bench_$m.err || { echo "bench $m failed"; tail -5 gpurun_out/c5f/bench_$m.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step']*1e3,1), 'us/step', round(d['value']), 'Msps')" gpurun_out/c5f/bench_$m.json $m
done
