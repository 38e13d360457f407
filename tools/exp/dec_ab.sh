#!/bin/bash
# A/B of the C5 audio FIR block shape (firDecFFKernel: GSDR_DEC_R outputs per lane x GSDR_DEC_THREADS):
# A/B libraries under tools/exp/_ablib/<variant>/ (GSDR_LIB), C5 sharded bench, interleaved rounds.
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/dec
for r in 1 2 3; do
  for v in base ${VARIANTS:-r2t256 r1t512 r2t128}; do
    if [ $v = base ]; then L=; else L=$PWD/tools/exp/_ablib/$v/libgpusdrpipeline.so; fi
    GSDR_LIB=$L timeout -k 10 120 python bench.py --workload c5 --steps 40 --warmup 5 --no-cpu-baseline > gpurun_out/dec/c5_${v}_$r.json 2>gpurun_out/dec/c5_${v}_$r.err || { echo "FAIL $v"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step']*1e3,1), 'us/step')" gpurun_out/dec/c5_${v}_$r.json $v
  done
done
