#!/bin/bash
# Round-4 session V: per-slot AM ring counts in the fused kernel (the tile-count race) - the chain,
# fused and shard tests, then the full GPU suite, smoke and the default bench. -> gpurun_out/r04v/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/r04v
mkdir -p "$OUT"
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_am_fused.py \
  tests/test_am_chain.py > "$OUT/tests_chain.log" 2>&1
rc=$?; echo "chain tests rc=$rc: $(tail -n 1 $OUT/tests_chain.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $OUT/gpu_tests.log)"
if [ $rc -ne 0 ]; then grep -E "FAILED|ERROR" "$OUT/gpu_tests.log" | head -20; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed"; tail -5 "$OUT/bench_default.err"; exit 1; }
echo "bench ok"; cut -c1-400 "$OUT/bench_default.json"
for wl in c3 c5; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${wl}_stats" -o run -- \
      python3 "$ROOT/bench.py" --workload $wl --steps 40 --warmup 2 --no-cpu-baseline --no-extras) > "$OUT/${wl}_prof.json" 2> "$OUT/${wl}_prof.err" || { echo "prof $wl failed"; exit 1; }
  python3 tools/kernel_trace_summary.py "$OUT/${wl}_stats" > "$OUT/${wl}_trace_summary.txt" || exit 1
  head -2 "$OUT/${wl}_trace_summary.txt"
done
echo "session v done"
