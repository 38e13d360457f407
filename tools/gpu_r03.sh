#!/bin/bash
# Round-3 GPU session (run on the box through gpurun): selected GPU tests, then the default bench.
#   MODE=tests|bench|all (default all); TESTS = pytest targets
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
MODE=${MODE:-all}
if [ "$MODE" != bench ]; then
  timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -v --maxfail=8 --timeout 300 --timeout-method thread \
    > gpurun_out/tests_r03.log 2>&1
  rc=$?
  echo "tests rc=$rc"; tail -3 gpurun_out/tests_r03.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
fi
if [ "$MODE" != tests ]; then
  timeout -k 10 600 python -u bench.py --steps 20 --warmup 5 > gpurun_out/bench_r03.log 2> gpurun_out/bench_r03.err
  rc=$?
  echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench_r03.log
  exit $rc
fi
