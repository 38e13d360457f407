#!/bin/bash
# Round-5 GPU session runner: tools/r05/session.sh NAME STEP [STEP ...] -> gpurun_out/r05<NAME>/
# Steps (each under its own time limit; a crash, abort or timeout ends the session so nothing else
# touches the GPU after a fault; a plain test failure does not):
#   tests      the full -m gpu suite                     stale     stale-LDS regression on the noz library
#   diag       ws_abort_diag.py on the diag library      smoke     __graft_entry__.smoke()
#   c5ab       C5 bench, 4-way vs 8-way int8 kernel (2 interleaved rounds)
#   bench      the default bench line                    prof      rocprofv3 kernel-trace of the default bench
#   hostfed    rocprofv3 kernel + memory-copy trace of the host-fed C5 leg
#   hostapi    the same with the HIP runtime API trace (which call blocks the host)
#   waits      hand-off wait profile of the C5 launch, 4-way and 8-way (waits library)
#   t:EXPR     the -m gpu tests selected by -k EXPR
#   ranks8     bench --gpus 8 --share-gpu --backend gloo (the driver's multi-rank path, 8 ranks on cuda:0)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
NAME=$1; shift
OUT=gpurun_out/r05$NAME
mkdir -p "$OUT"
export TMPDIR=/tmp

step() {  # step <name> <timeout> <cmd...>
  local name=$1 limit=$2; shift 2
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "$OUT/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc"
  tail -n 6 "$OUT/$name.log" | cut -c1-400
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "FATAL: $name exited $rc; stopping the session"; exit $rc
  fi
  return 0
}

for s in "$@"; do
  case "$s" in
    tests) step tests 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread ;;
    stale) GSDR_LIB=$PWD/tools/exp/_ablib/noz/libgpusdrpipeline.so step stale_noz 300 python -u -m pytest -q \
             -p no:cacheprovider --timeout 120 --timeout-method thread tests/test_am_fused.py -k stale_lds ;;
    diag) GSDR_LIB=$PWD/tools/exp/_ablib/diag/libgpusdrpipeline.so step ws_abort_diag 300 python3 -u tools/exp/ws_abort_diag.py ;;
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" ;;
    c5ab) for r in 1 2; do
            step c5_ws4_$r 300 python -u bench.py --workload c5 --no-extras --no-cpu-baseline --steps 60 --warmup 5
            step c5_ws8_$r 300 python -u bench.py --workload c5 --no-extras --no-cpu-baseline --steps 60 --warmup 5 --kernel-policy 64
          done ;;
    bench) step bench_default 600 python -u bench.py ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof" -o run -- \
            python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline ;;
    hostfed) step hostfed 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d "$OUT/hostfed" -o run -- \
               python3 tools/exp/host_fed_probe.py ;;
    hostapi) step hostapi 300 rocprofv3 --hip-runtime-trace --kernel-trace --memory-copy-trace --output-format csv \
               -d "$OUT/hostapi" -o run -- python3 tools/exp/host_fed_probe.py ;;
    waits) GSDR_LIB=$PWD/tools/exp/_ablib/waits/libgpusdrpipeline.so step c5_waits_ws4 300 python3 -u tools/exp/c5_waits_probe.py
           GSDR_LIB=$PWD/tools/exp/_ablib/waits/libgpusdrpipeline.so step c5_waits_ws8 300 python3 -u tools/exp/c5_waits_probe.py --ws8 ;;
    t:*) step "test_${s#t:}" 600 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "${s#t:}" ;;
    ranks8) step ranks8 900 python -u bench.py --gpus 8 --share-gpu --backend gloo --steps 5 --warmup 2 ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "session $NAME done"
