#!/bin/bash
# Round-6 GPU session runner: tools/r06/session.sh NAME STEP [STEP ...] -> gpurun_out/r06<NAME>/
# Steps (each under its own time limit; a crash, abort or timeout ends the session so nothing else
# touches the GPU after a fault; a plain test failure does not):
#   tests      the full -m gpu suite                     smoke     __graft_entry__.smoke()
#   t:EXPR     the -m gpu tests selected by -k EXPR      f:FILE    one test file (tests/FILE.py), -m gpu
#   bench      the default bench line                    prof      rocprofv3 kernel-trace of the default bench
#   c5n2       bench --workload c5 --gpus 2 --share-gpu --backend gloo (the multi-rank C5 step, 4-way kernel)
#   ranks8     bench --gpus 8 --share-gpu --backend gloo (the driver's multi-rank path, 8 ranks on cuda:0)
#   py:SCRIPT  python3 -u SCRIPT (a probe under tools/)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
NAME=$1; shift
OUT=gpurun_out/r06$NAME
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <timeout> <cmd...>
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 6 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ] && [ $rc -ne 5 ]; then  # 5: pytest collected nothing
    echo "FATAL: $name exited $rc; stopping the session"; exit $rc
  fi
  return 0
}

PYT="python -u -m pytest -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread"
for s in "$@"; do
  case "$s" in
    tests) step tests 900 $PYT tests ;;
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench_default 600 python -u bench.py ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
            python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
    c5n2) step c5_n2 420 python -u bench.py --workload c5 --gpus 2 --share-gpu --backend gloo --no-extras \
            --no-cpu-baseline --steps 20 --warmup 3 ;;
    ranks8) step ranks8 900 python -u bench.py --gpus 8 --share-gpu --backend gloo --steps 5 --warmup 2 ;;
    t:*) step "test_${s#t:}" 600 $PYT tests -k "${s#t:}" ;;
    f:*) step "file_${s#f:}" 600 $PYT "tests/${s#f:}.py" -v ;;
    py:*) step "py_$(basename "${s#py:}" .py)" 600 python3 -u "${s#py:}" ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session $NAME done"
