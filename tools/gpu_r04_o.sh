#!/bin/bash
# Round-4 session O: is C5 slower than at 20:00 (0.170 ms launch)? Interleaved C5 benches of the
# current library, the r04 profile-set kernel source (old) and the prefetch / poll variants; no
# profiler before them. -> gpurun_out/r04o/
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04o
mkdir -p "$OUT"
VARS=${VARS:-"old pf2 pf3p"}
for r in 1 2 3; do
  for v in base $VARS; do
    if [ $v = base ]; then L=; else L=$PWD/tools/exp/_ablib/$v/libgpusdrpipeline.so; fi
    GSDR_LIB=$L timeout -k 10 120 python3 bench.py --workload c5 --steps 40 --warmup 5 --no-cpu-baseline --no-extras \
      > "$OUT/c5_${v}_$r.json" 2> "$OUT/c5_${v}_$r.err" || { echo "FAIL $v"; exit 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], round(d['ms_per_step']*1e3,1), 'us/step, launch', round(r['avg_launch_ms']*1e3,1), 'us')" "$OUT/c5_${v}_$r.json" $v
  done
done
echo "session o done"
