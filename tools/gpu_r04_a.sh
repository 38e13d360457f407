#!/bin/bash
# Round-4 session A: (1) the C3 epilogue question (AM-epilogue launch vs complex launch + AM pass),
# HIP events and a rocprofv3 kernel trace; (2) the node-path leg under a kernel trace; (3) the FFT
# kernel's in-kernel clock from wave stamps after 2.5 s of back-to-back launches (per attribution
# variant). -> gpurun_out/r04a/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/r04a
mkdir -p "$OUT"
timeout -k 10 300 python3 -u tools/exp/c3_epilogue_probe.py > "$OUT/epilogue.log" 2>&1
rc=$?; echo "epilogue rc=$rc"; cat "$OUT/epilogue.log" | tail -6; [ $rc -eq 0 ] || exit $rc
(cd /tmp && ROUNDS=2 timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/epi_stats" -o run -- \
    python3 "$ROOT/tools/exp/c3_epilogue_probe.py") > "$OUT/epi_prof.log" 2>&1
rc=$?; echo "epi prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/epi_prof.log"; exit $rc; }
python3 tools/kernel_trace_summary.py "$OUT/epi_stats" > "$OUT/epi_trace_summary.txt" 2>&1 || true
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/nodes_stats" -o run -- \
    python3 "$ROOT/tools/exp/c3_nodes_probe.py") > "$OUT/nodes_prof.log" 2>&1
rc=$?; echo "nodes prof rc=$rc"; [ $rc -eq 0 ] || { tail -5 "$OUT/nodes_prof.log"; exit $rc; }
python3 tools/kernel_trace_summary.py "$OUT/nodes_stats" > "$OUT/nodes_trace_summary.txt" 2>&1 || true
FFT_BENCH_STAMPS=1 timeout -k 10 300 tools/exp/_build_fft/fft_bench > "$OUT/stamps.log" 2>&1
rc=$?; echo "stamps rc=$rc"; cat "$OUT/stamps.log"; [ $rc -eq 0 ] || exit $rc
echo "session A done"
