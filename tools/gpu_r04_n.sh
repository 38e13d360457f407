#!/bin/bash
# Round-4 session N: C5 consumer A-fragment prefetch depth (GSDR_WS_PF) A/B - fused-chain parity per
# variant library, then interleaved C5 bench rounds. -> gpurun_out/r04n/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04n
mkdir -p "$OUT"
VARS=${VARS:-"pf2 pf3 pf4 p1 pf3p"}
for v in ${TVARS:-pf3p pf4}; do
  GSDR_LIB=$PWD/tools/exp/_ablib/$v/libgpusdrpipeline.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 \
    --timeout-method thread tests/test_am_fused.py > "$OUT/tests_$v.log" 2>&1
  rc=$?; echo "tests $v rc=$rc: $(tail -n 1 $OUT/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for r in 1 2; do
  for v in base $VARS; do
    if [ $v = base ]; then L=; else L=$PWD/tools/exp/_ablib/$v/libgpusdrpipeline.so; fi
    GSDR_LIB=$L timeout -k 10 120 python3 bench.py --workload c5 --steps 40 --warmup 5 --no-cpu-baseline --no-extras \
      > "$OUT/c5_${v}_$r.json" 2> "$OUT/c5_${v}_$r.err" || { echo "FAIL $v"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], round(d['ms_per_step']*1e3,1), 'us/step', d['roofline'].get('achieved'), d['roofline'].get('unit'))" "$OUT/c5_${v}_$r.json" $v
  done
done
echo "session n done"
