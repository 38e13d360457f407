#!/bin/bash
# Round-4 session G: the full GPU suite + smoke, the default bench (C3 + extras), then the r04 profile
# set (kernel-trace stats, FETCH/WRITE PMC, SQ passes) of C3, C4s, C5, C2. -> gpurun_out/r04g/, r04prof/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04q
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $OUT/gpu_tests.log)"
if [ $rc -ne 0 ]; then grep -E "FAILED|ERROR" "$OUT/gpu_tests.log" | head -20; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed"; tail -5 "$OUT/bench_default.err"; exit 1; }
echo "bench ok"; cut -c1-600 "$OUT/bench_default.json"
bash tools/prof_r04.sh c3 c5
