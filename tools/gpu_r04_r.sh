#!/bin/bash
# Round-4 session R: does the profiler change the kernels' speed? The same bench command without,
# under rocprofv3 --kernel-trace --stats, and without again, for C5 and C3. -> gpurun_out/r04r/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$(pwd)
export TMPDIR=/tmp
OUT=$ROOT/gpurun_out/r04r
mkdir -p "$OUT"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step']*1e3,1), 'us/step, launch', round(r['avg_launch_ms']*1e3,1), 'us')" "$1" "$2"; }
for wl in c5 c3; do
  timeout -k 10 200 python3 bench.py --workload $wl --steps 40 --warmup 5 --no-cpu-baseline --no-extras > "$OUT/${wl}_plain1.json" 2>/dev/null || exit 1
  show "$OUT/${wl}_plain1.json" "$wl plain"
  (cd /tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/${wl}_prof" -o run -- \
      python3 "$ROOT/bench.py" --workload $wl --steps 40 --warmup 5 --no-cpu-baseline --no-extras) > "$OUT/${wl}_prof.json" 2> "$OUT/${wl}_prof.err" || exit 1
  show "$OUT/${wl}_prof.json" "$wl under rocprof"
  python3 tools/kernel_trace_summary.py "$OUT/${wl}_prof" | head -3
  timeout -k 10 200 python3 bench.py --workload $wl --steps 40 --warmup 5 --no-cpu-baseline --no-extras > "$OUT/${wl}_plain2.json" 2>/dev/null || exit 1
  show "$OUT/${wl}_plain2.json" "$wl plain"
done
echo "session r done"
