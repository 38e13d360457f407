#!/bin/bash
# Round-3 closing GPU session: the full GPU suite and smoke(), the default bench (C3 + extras), then
# rocprofv3 kernel-trace stats of the C3 and C5 bench commands (kept under gpurun_out/r03final/).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/r03final
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $OUT/gpu_tests.log)"
if [ $rc -ne 0 ]; then grep -E "FAILED|ERROR" "$OUT/gpu_tests.log" | head -20; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed"; tail -5 "$OUT/bench_default.err"; exit 1; }
echo "bench ok"
for WL in c3 c5; do
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${WL}_stats" -o run -- \
      python3 "$ROOT/bench.py" --workload $WL --steps 40 --warmup 2 --no-cpu-baseline --no-extras) > "$OUT/${WL}_prof.log" 2>&1
  rc=$?; echo "rocprof $WL rc=$rc"
  if [ $rc -ne 0 ]; then tail -5 "$OUT/${WL}_prof.log"; exit $rc; fi
  python3 tools/kernel_trace_summary.py "$OUT/${WL}_stats" > "$OUT/${WL}_trace_summary.txt" 2>&1 || true
done
echo "final session done"
