#!/bin/bash
# Round-4 session X: the multi-rank bench protocol after the pre-settle barrier (2 gloo ranks sharing
# cuda:0). -> gpurun_out/r04x/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04x
mkdir -p "$OUT"
for wl in c3 c5; do
  timeout -k 10 300 python3 -u bench.py --gpus 2 --share-gpu --backend gloo --workload $wl --steps 10 --warmup 3 \
    --no-extras > "$OUT/bench_${wl}_g2_gloo.json" 2> "$OUT/bench_${wl}_g2_gloo.err"
  rc=$?; echo "$wl rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_${wl}_g2_gloo.err"; exit $rc; }
  cut -c1-300 "$OUT/bench_${wl}_g2_gloo.json"
done
echo "session x done"
