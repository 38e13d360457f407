#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/ws
for r in 1 2; do
  for v in base cons1 prod1; do
    if [ $v = base ]; then L=; else L=$PWD/tools/exp/_ablib/$v/libgpusdrpipeline.so; fi
    GSDR_LIB=$L timeout -k 10 120 python bench.py --workload c5 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/ws/c5_${v}_$r.json 2>gpurun_out/ws/c5_${v}_$r.err || { echo "FAIL $v"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'])" gpurun_out/ws/c5_${v}_$r.json $v
  done
done
