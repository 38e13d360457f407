#!/bin/bash
# Round-4 session S: the bench after moving the GC collection in front of the settle (no idle gap
# before the timed steps): C5 and C3 alone, then the default run. -> gpurun_out/r04s/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04s
mkdir -p "$OUT"
show() { python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step']*1e3,1), 'us/step, launch', round(r['avg_launch_ms']*1e3,1), 'us, frac', round(r['frac'],3))" "$1" "$2"; }
for wl in c5 c3; do
  timeout -k 10 200 python3 bench.py --workload $wl --steps 40 --warmup 5 --no-cpu-baseline --no-extras > "$OUT/${wl}.json" 2>/dev/null || exit 1
  show "$OUT/${wl}.json" "$wl"
done
timeout -k 10 600 python3 -u bench.py > "$OUT/bench_default.json" 2> "$OUT/bench_default.err" || { echo "bench failed"; tail -5 "$OUT/bench_default.err"; exit 1; }
show "$OUT/bench_default.json" "default c3"
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for k,v in d['extras'].items():
    print(k, {kk: v.get(kk) for kk in ('ms_per_step','avg_launch_ms','frac')})
" "$OUT/bench_default.json"
echo "session s done"
