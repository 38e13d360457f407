#!/bin/bash
# Round-4 session U (closing, final tree): the full GPU suite + smoke, the default bench, and a
# kernel-trace profile of C3 and C5. -> gpurun_out/r04u/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/r04u
mkdir -p "$OUT"
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
echo "session u done"
