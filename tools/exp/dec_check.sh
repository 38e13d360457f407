#!/bin/bash
# Parity tests of the audio-FIR block-shape A/B libraries, then the C5 A/B (tools/exp/dec_ab.sh).
set -u
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for v in ${VARIANTS:-r2t256 r1t512 r2t128}; do
  GSDR_LIB=$PWD/tools/exp/_ablib/$v/libgpusdrpipeline.so timeout -k 10 200 python -m pytest tests/test_gpu_parity.py tests/test_am_chain.py \
    -m gpu -q -k "phase_pair or chain" --timeout 120 --timeout-method thread > gpurun_out/dec_tests_$v.log 2>&1
  rc=$?
  echo "$v tests rc=$rc: $(tail -1 gpurun_out/dec_tests_$v.log)"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
done
bash tools/exp/dec_ab.sh
