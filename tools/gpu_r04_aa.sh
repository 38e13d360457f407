#!/bin/bash
# Round-4 session AA: hand-off polls without s_sleep (GSDR_WS_SLEEP=0) - fused / chain tests on the
# variant, then interleaved C5 benches against the default (s_sleep 1). -> gpurun_out/r04aa/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04aa
mkdir -p "$OUT"
V=$PWD/tools/exp/_ablib/sl0/libgpusdrpipeline.so
GSDR_LIB=$V timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_am_fused.py \
  tests/test_am_chain.py > "$OUT/tests_sl0.log" 2>&1
rc=$?; echo "sl0 tests rc=$rc: $(tail -n 1 $OUT/tests_sl0.log)"; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in base sl0; do
    if [ $v = base ]; then L=; else L=$V; fi
    GSDR_LIB=$L timeout -k 10 120 python3 bench.py --workload c5 --steps 40 --warmup 5 --no-cpu-baseline --no-extras \
      > "$OUT/c5_${v}_$r.json" 2> "$OUT/c5_${v}_$r.err" || { echo "FAIL $v"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step']*1e3,1), 'us/step, launch', round(r['avg_launch_ms']*1e3,1), 'us')" "$OUT/c5_${v}_$r.json" $v
  done
done
echo "session aa done"
