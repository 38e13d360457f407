#!/bin/bash
# Round-4 session M: LDS counters of the fused C5 kernel (is the consumer side LDS-bound?).
# -> gpurun_out/r04prof/c5_sq2, c5_sq3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/r04prof
mkdir -p "$OUT"
WL=c5
run() {
  local d=$1; shift
  echo "=== $d ($(date +%T))"
  (cd /tmp && timeout -k 10 240 rocprofv3 "$@" --output-format csv -d "$OUT/$d" -o run -- \
      python3 "$ROOT/bench.py" --workload "$WL" --steps 10 --warmup 2 --no-cpu-baseline --no-extras) > "$OUT/$d.log" 2>&1
  local rc=$?
  echo "=== $d rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 20 "$OUT/$d.log"; exit $rc; fi
}
run c5_sq2 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE
run c5_sq3 --pmc SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE
echo "session m done"
bash tools/gpu_r04_n.sh
