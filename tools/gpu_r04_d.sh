#!/bin/bash
# Round-4 session D: the WS abort root-cause diagnostic (tools/exp/ws_abort_diag.py on the
# GSDR_WS_DIAG build). -> gpurun_out/r04d/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04d
mkdir -p "$OUT"
GSDR_LIB=$PWD/cuda-sdr_amd/lib_diag/libgpusdrpipeline.so timeout -k 10 180 python3 -u tools/exp/ws_abort_diag.py > "$OUT/ws_abort_diag.log" 2>&1
rc=$?; echo "ws diag rc=$rc"; cat "$OUT/ws_abort_diag.log" | grep -v amdgpu.ids; exit $rc
