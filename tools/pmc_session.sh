#!/bin/bash
# rocprofv3 PMC passes over a short bench run (one counter group per pass, kernel trace only).
# Usage: bash tools/pmc_session.sh [workload]   -> gpurun_out/pmc_<group>/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
WL=${1:-c2}
OUT=gpurun_out
mkdir -p "$OUT"
pass() {  # pass <name> <counters...>
  local name=$1; shift
  echo "=== pmc $name ($(date +%T))"
  timeout -k 10 300 rocprofv3 --pmc "$@" --output-format csv -d "$OUT/pmc_$name" -o run -- \
      python bench.py --workload "$WL" --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/pmc_$name.log" 2>&1
  local rc=$?
  echo "=== pmc $name rc=$rc"
  if [ $rc -ne 0 ]; then tail -n 20 "$OUT/pmc_$name.log"; exit $rc; fi
}
pass fetch FETCH_SIZE
pass write WRITE_SIZE
pass sq1 SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES
pass sq2 SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM
python tools/pmc_traffic.py "$WL" "$OUT/pmc_fetch" "$OUT/pmc_write" "$OUT/pmc_traffic.json"
echo "pmc session done"
