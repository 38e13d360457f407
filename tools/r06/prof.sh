#!/bin/bash
# Round-6 profile session on one MI355X: per workload a kernel-trace --stats run of bench.py (the per-kernel
# average durations the bench's HIP-event roofline must agree with), FETCH_SIZE / WRITE_SIZE PMC passes
# (HBM bytes per launch, tools/pmc_traffic.py) and SQ passes (waits / MFMA / LDS), each pass its own run.
# Usage: bash tools/r06/prof.sh NAME [workloads...]   -> gpurun_out/r06prof_NAME/   (POLICY=<flags> for A/B)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
ROOT=$(pwd)
export TMPDIR=/tmp
NAME=$1; shift
OUT=$ROOT/gpurun_out/r06prof_$NAME
mkdir -p "$OUT"
WLS=${*:-c3 c4s c5 c2}
run() {  # run <dir> <rocprof args...> : rocprofv3 <args> over a short bench run
  local d=$1; shift
  echo "=== $d ($(date +%T))"
  (cd /tmp && timeout -k 10 240 rocprofv3 "$@" --output-format csv -d "$OUT/$d" -o run -- \
      python3 "$ROOT/bench.py" --workload "$WL" --steps ${STEPS:-10} --warmup 2 --no-cpu-baseline --no-extras \
      --kernel-policy ${POLICY:-0}) > "$OUT/$d.log" 2>&1
  local rc=$?
  echo "=== $d rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 20 "$OUT/$d.log"; exit $rc; fi
}
for WL in $WLS; do
  STEPS=40 run "${WL}_stats" --kernel-trace --stats
  python3 tools/kernel_trace_summary.py "$OUT/${WL}_stats" > "$OUT/${WL}_trace_summary.txt" || exit 1
  if [ -z "${NO_TRAFFIC:-}" ]; then
    run "${WL}_fetch" --pmc FETCH_SIZE
    run "${WL}_write" --pmc WRITE_SIZE
    python3 tools/pmc_traffic.py "$WL" "$OUT/${WL}_fetch" "$OUT/${WL}_write" "$OUT/${WL}_traffic.json" || exit 1
  fi
  run ${WL}_sq1 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE
  run ${WL}_sq2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE
  python3 tools/pmc_sq.py "$OUT/${WL}_sq1" "$OUT/${WL}_sq2" --json "$OUT/pmc_sq_${WL}.json" > "$OUT/pmc_sq_${WL}.txt" || exit 1
done
echo "profile session done"
