set -u
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/c5sq
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_fft_fir.py -m gpu -q -x --timeout 100 --timeout-method thread -k unaligned > gpurun_out/unaligned_test.log 2>&1 || exit 1
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  (cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload c5 --steps 5 --warmup 2 --no-cpu-baseline --no-extras) > $OUT/p$i.log 2>&1 || exit 2
done
python3 tools/pmc_sq.py $OUT/p1 $OUT/p2 --json $OUT/sq.json > $OUT/sq.txt
echo done
