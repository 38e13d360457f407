#!/bin/bash
# Round-4 session AE (closing): the stale-LDS regression test against a library built without the
# ring zeroing (expected to fail) and the product library, then the full GPU suite, smoke and the
# default bench on the final tree. -> gpurun_out/r04ae/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04ae
mkdir -p "$OUT"
GSDR_LIB=$PWD/tools/exp/_ablib/noz/libgpusdrpipeline.so timeout -k 10 300 python3 -u -m pytest -q --timeout 120 \
  --timeout-method thread tests/test_am_fused.py -k stale_lds > "$OUT/stale_lds_without_zeroing.log" 2>&1
echo "without ring zeroing (expected to fail): rc=$? $(tail -n 1 $OUT/stale_lds_without_zeroing.log)"
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1
rc=$?; echo "tests rc=$rc: $(tail -1 $OUT/gpu_tests.log)"
if [ $rc -ne 0 ]; then grep -E "FAILED|ERROR" "$OUT/gpu_tests.log" | head -20; exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || { echo "smoke failed"; tail -5 "$OUT/smoke.log"; exit 1; }
tail -1 "$OUT/smoke.log"
timeout -k 10 600 python -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed"; tail -5 "$OUT/bench_default.err"; exit 1; }
echo "bench ok"; cut -c1-300 "$OUT/bench_default.json"
echo "session ae done"
