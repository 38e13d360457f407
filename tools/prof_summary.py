#!/usr/bin/env python3
"""Summarise a rocprofv3 --kernel-trace CSV per (kernel, grid size): calls, mean/min/max ns.

The bench launches the same FIR kernel twice per step (bulk + halo head), so the per-name
average of --stats mixes them; grouping by grid size separates the dominant bulk launch."""
import collections
import csv
import json
import sys


def main(path, out=None):
    groups = collections.defaultdict(list)
    with open(path) as f:
        for row in csv.DictReader(f):
            key = (row["Kernel_Name"], int(row["Grid_Size_X"]), int(row["LDS_Block_Size"]),
                   int(row["VGPR_Count"]), int(row["SGPR_Count"]))
            groups[key].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    rows = []
    for (name, grid, lds, vgpr, sgpr), d in sorted(groups.items(), key=lambda kv: -sum(kv[1])):
        d_sorted = sorted(d)
        rows.append({"kernel": name, "grid_threads": grid, "lds_bytes": lds, "vgpr": vgpr, "sgpr": sgpr,
                     "calls": len(d), "mean_ns": sum(d) / len(d), "median_ns": d_sorted[len(d) // 2],
                     "min_ns": d_sorted[0], "max_ns": d_sorted[-1]})
    text = json.dumps(rows, indent=1)
    if out:
        with open(out, "w") as f:
            f.write(text + "\n")
    print(text)


if __name__ == "__main__":
    main(*sys.argv[1:])
