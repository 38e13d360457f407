#!/bin/bash
# Round-4 session K: the fused C5 launch's hand-off wait profile (GSDR_WS_WAITS build). -> gpurun_out/r04k/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04k
mkdir -p "$OUT"
GSDR_LIB=$PWD/cuda-sdr_amd/lib_waits/libgpusdrpipeline.so timeout -k 10 180 python3 -u tools/exp/c5_waits_probe.py > "$OUT/c5_waits.log" 2>&1
rc=$?; echo "c5 waits rc=$rc"; grep -v amdgpu.ids "$OUT/c5_waits.log" | tail -8; exit $rc
