#!/usr/bin/env python3
"""Per-kernel means of every counter in rocprofv3 --pmc output directories.

Usage: pmc_sq.py <dir> [<dir> ...] [--json out.json]
Prints, for each kernel (and grid size), the mean per-dispatch value of each counter collected,
and writes them as JSON when asked. SQ cycle counters are in quad-cycles except
SQ_VALU_MFMA_BUSY_CYCLES (MI355X_MICROARCH.md, rocprofv3 PMC slots / cycle constants).
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def main(argv):
    out = None
    if "--json" in argv:
        i = argv.index("--json")
        out = argv[i + 1]
        argv = argv[:i] + argv[i + 2:]
    acc = defaultdict(lambda: defaultdict(list))
    for d in argv:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for r in csv.DictReader(f):
                    key = f'{r["Kernel_Name"][:90]} grid={r.get("Grid_Size") or r.get("Grid_Size_X")}'
                    acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {k: {c: sum(v) / len(v) for c, v in sorted(cs.items())} for k, cs in acc.items()}
    for k, cs in res.items():
        print(k)
        for c, v in cs.items():
            print(f"    {c:32s} {v:16.1f}")
    if out:
        with open(out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main(sys.argv[1:])
