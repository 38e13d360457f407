#!/bin/bash
# One GPU-box session: parity tests, smoke, a short bench and a rocprofv3 kernel-trace profile.
# Every GPU step has its own time limit; a crash/abort/timeout (exit status other than 0 or a
# plain test failure) ends the session so nothing else touches the GPU after a fault.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <timeout> <cmd...>
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 25 "$OUT/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "FATAL: $name exited $rc; stopping the session"; exit $rc
  fi
  return 0
}

WHAT=${1:-all}
case "$WHAT" in
  *tests*|all) step pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider ;;&
  *smoke*|all) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;&
  *bench*|all) step bench 600 python bench.py --steps 30 --warmup 5 ;;&
  *prof*|all)  step rocprof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
                  python bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;&
  *pmc*|all)   step pmc 1100 bash tools/pmc_session.sh c2 ;;&
  *) ;;
esac
echo "session done"
