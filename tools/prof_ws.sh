#!/bin/bash
# rocprofv3 kernel-trace summaries of the C3 and C5 bench workloads (wave-specialised kernels).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out; mkdir -p $OUT
for wl in c3 c5 c2; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$wl -o run -- \
    python3 bench.py --workload $wl --steps 10 --warmup 2 --no-cpu-baseline > $OUT/prof_$wl.log 2>&1
  rc=$?; echo "== $wl rc=$rc"; tail -n 1 $OUT/prof_$wl.log | cut -c1-300
  [ $rc -ne 0 ] && exit $rc
  f=$(find $OUT/prof_$wl -name "*kernel_stats.csv" | head -1); [ -n "$f" ] && cut -d, -f1-8 "$f" | head -8
done
