#!/bin/bash
# Round-4 session AC: rate of the intermittent short-filter executor failure - the first test files
# of the suite, 4 runs with the product library and 4 with one built at r03's poll / prefetch
# settings (GSDR_WS_PF=1 GSDR_WS_POLL=0). -> gpurun_out/r04ac/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04ac
mkdir -p "$OUT"
V=$PWD/tools/exp/_ablib/r03poll/libgpusdrpipeline.so
for r in 1 2 3 4; do
  for v in base r03poll; do
    if [ $v = base ]; then L=; else L=$V; fi
    GSDR_LIB=$L timeout -k 10 200 python3 -u -m pytest -q --timeout 120 --timeout-method thread -m gpu \
      tests/test_abi_exports.py tests/test_am_chain.py -p no:cacheprovider > "$OUT/run_${v}_$r.log" 2>&1
    rc=$?
    echo "$v run $r rc=$rc: $(tail -n 1 $OUT/run_${v}_$r.log)"
    [ $rc -le 1 ] || exit $rc
  done
done
echo "session ac done"
