#!/bin/bash
# Round-4 session L: paired row-group transposition A/B; the multi-rank protocol on one GPU (2 gloo ranks sharing cuda:0, halos staged
# through host memory) for C3 and C5, and the C5 executor modes. -> gpurun_out/r04l/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04l
mkdir -p "$OUT"
timeout -k 10 300 tools/exp/_build_fft_ab/fft_bench > "$OUT/tpair_ab.log" 2>&1
rc=$?; echo "tpair ab rc=$rc"; cat "$OUT/tpair_ab.log"; [ $rc -eq 0 ] || exit $rc
for wl in c3 c5; do
  timeout -k 10 300 python3 -u bench.py --gpus 2 --share-gpu --backend gloo --workload $wl --steps 10 --warmup 3 \
      --no-extras > "$OUT/bench_${wl}_g2_gloo.json" 2> "$OUT/bench_${wl}_g2_gloo.err"
  rc=$?; echo "$wl g2 rc=$rc"; cut -c1-300 "$OUT/bench_${wl}_g2_gloo.json"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_${wl}_g2_gloo.err"; exit $rc; }
done
for m in resident chunked; do
  timeout -k 10 300 python3 -u bench.py --workload c5 --c5-mode $m --steps 20 --warmup 3 --no-extras --no-cpu-baseline \
      > "$OUT/bench_c5_$m.json" 2> "$OUT/bench_c5_$m.err"
  rc=$?; echo "c5 $m rc=$rc"; cut -c1-300 "$OUT/bench_c5_$m.json"; [ $rc -eq 0 ] || { tail -5 "$OUT/bench_c5_$m.err"; exit $rc; }
done
