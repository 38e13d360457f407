#!/bin/bash
# Round-4 session T: tile i-1 reduction interleaved with tile i MFMAs (int8 WS consumers) - C5 chain / fused / shard tests and the abort
# tests on the new default, then interleaved C5 benches against the sequential reduction (noil).
# -> gpurun_out/r04p/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04t
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_am_fused.py \
  tests/test_am_chain.py > "$OUT/tests_chain.log" 2>&1
rc=$?; echo "chain tests rc=$rc: $(tail -n 1 $OUT/tests_chain.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_shard_gpu.py \
  tests/test_gpu_parity.py -k "abort or c5 or chain or am" > "$OUT/tests_shard.log" 2>&1
rc=$?; echo "shard/abort tests rc=$rc: $(tail -n 1 $OUT/tests_shard.log)"; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  for v in base noil; do
    if [ $v = base ]; then L=; else L=$PWD/tools/exp/_ablib/$v/libgpusdrpipeline.so; fi
    GSDR_LIB=$L timeout -k 10 120 python3 bench.py --workload c5 --steps 40 --warmup 5 --no-cpu-baseline --no-extras \
      > "$OUT/c5_${v}_$r.json" 2> "$OUT/c5_${v}_$r.err" || { echo "FAIL $v"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step']*1e3,1), 'us/step, launch', round(r['avg_launch_ms']*1e3,1), 'us')" "$OUT/c5_${v}_$r.json" $v
  done
done
echo "session p done"
