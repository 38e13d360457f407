#!/bin/bash
# A/B of the one-wave-per-SIMD prefetching FFT kernels against the committed 8-wave kernel
# (tools/exp/run_fft_variants.sh), then the FFT parity tests and the C3 / C4 bench lines on the
# rebuilt library. Each GPU step has its own time limit; the first failure ends the run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pf; mkdir -p $OUT
run() { local name=$1 lim=$2; shift 2; timeout -k 10 "$lim" "$@" > "$OUT/$name.log" 2>&1; local rc=$?;
        echo "== $name rc=$rc"; tail -n ${TAILN:-4} "$OUT/$name.log" | cut -c1-400
        if [ $rc -ne 0 ]; then echo "FATAL $name"; exit $rc; fi; }
TAILN=12 run ab 300 bash tools/exp/run_fft_variants.sh run
run pytest_fft 600 python -u -m pytest tests/test_fft_fir.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider
run bench_c3 300 python bench.py --no-cpu-baseline
run bench_c4 300 python bench.py --workload c4 --no-cpu-baseline
echo "pf done"
