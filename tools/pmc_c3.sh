set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE"; do
  name=$(echo $grp | cut -c1-12 | tr -d ' ')
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmcc3_$name -o run -- python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/pmcc3_$name.log 2>&1 || exit 1
done
echo done
