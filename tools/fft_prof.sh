#!/bin/bash
# FFT FIR iteration: parity tests, C3 bench + kernel trace, and two SQ PMC passes on C3.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out; mkdir -p $OUT
export TMPDIR=/tmp
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
        echo "== $name rc=$rc"; tail -n ${TAILN:-4} "$OUT/$name.log" | cut -c1-1800
        if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "FATAL $name"; exit $rc; fi; }
TAILN=30 run pytest_fft 400 python -u -m pytest tests/test_fft_fir.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider
run bench_c3 200 python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline
run rocprof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_c3" -o run -- python bench.py --workload c3 --steps 10 --warmup 2 --no-cpu-baseline
find $OUT/prof_c3 -name "*kernel_stats.csv" -exec head -3 {} \;
if [ "${PMC:-1}" = 1 ]; then
i=0
for grp in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  run pmc$i 120 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc_fft$i -o run -- python bench.py --workload c3 --steps 3 --warmup 1 --no-cpu-baseline
done
python tools/pmc_sq.py $OUT/pmc_fft1 $OUT/pmc_fft2 | grep -A40 firFft | head -40
fi
