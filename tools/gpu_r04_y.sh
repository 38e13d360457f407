#!/bin/bash
# Round-4 session Y: the chain executor's short-filter cases repeated (intermittent U failure hunt).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r04y
GSDR_LIB=${GSDR_LIB:-} timeout -k 10 400 python3 -u tools/exp/chain_stress.py ${REPS:-40} > gpurun_out/r04y/chain_stress${TAG:-}.log 2>&1
rc=$?; tail -5 gpurun_out/r04y/chain_stress${TAG:-}.log; grep "bad" gpurun_out/r04y/chain_stress${TAG:-}.log | head -10; exit $rc
