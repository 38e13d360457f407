#!/usr/bin/env python3
"""Per-kernel launch-duration summary of a rocprofv3 --kernel-trace CSV run directory: count, mean,
median, min, max, and the mean without the first launch of each kernel (a cold first launch -
LDS attribute setup, first touch of the code object - inflates the plain mean of short runs).
Usage: kernel_trace_summary.py <rocprof output dir>"""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main(d):
    paths = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    if not paths:
        print("no kernel_trace.csv under", d, file=sys.stderr)
        return 1
    dur = defaultdict(list)
    for p in paths:
        with open(p) as f:
            for r in csv.DictReader(f):
                dur[r["Kernel_Name"]].append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"])))
    print(f"{'kernel':<70} {'n':>4} {'mean_us':>9} {'median_us':>9} {'min_us':>8} {'max_us':>8} {'mean_wo_first':>13}")
    for name, v in sorted(dur.items(), key=lambda kv: -sum(x for _, x in kv[1])):
        v.sort()
        xs = [x / 1e3 for _, x in v]
        rest = xs[1:] or xs
        print(f"{name[:70]:<70} {len(xs):>4} {statistics.mean(xs):>9.1f} {statistics.median(xs):>9.1f} "
              f"{min(xs):>8.1f} {max(xs):>8.1f} {statistics.mean(rest):>13.1f}")
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1]))
