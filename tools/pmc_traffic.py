#!/usr/bin/env python3
"""HBM bytes per launch of the dominant (largest-grid) FIR kernel from rocprofv3 --pmc runs.

Usage: pmc_traffic.py <workload> <fetch_dir> <write_dir> [out.json]
The two directories hold separate `rocprofv3 --pmc FETCH_SIZE` and `--pmc WRITE_SIZE` runs
(the counters do not fit one pass on gfx950, MI355X_MICROARCH.md "rocprofv3 PMC slots").
FETCH_SIZE / WRITE_SIZE are in KiB. On gfx950 FETCH_SIZE counts 64 B per 128-B request of a wide
coalesced stream (the guide's 1/2 correction for 16-B-per-lane loads); the correction is applied
and both raw values are kept so the judgement can be redone.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter):
    rows = []
    for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(path) as f:
            for r in csv.DictReader(f):
                if r.get("Counter_Name") != counter:
                    continue
                grid = int(r.get("Grid_Size") or r.get("Grid_Size_X") or 0)
                rows.append((r["Kernel_Name"], grid, float(r["Counter_Value"])))
    return rows


def dominant(rows):
    fir = [r for r in rows if "firLdsKernel" in r[0] or "fir" in r[0].lower()]
    if not fir:
        return None
    gmax = max(r[1] for r in fir)
    vals = [r[2] for r in fir if r[1] == gmax]
    name = next(r[0] for r in fir if r[1] == gmax)
    return {"kernel": name, "grid_threads": gmax, "launches": len(vals), "mean_kib": sum(vals) / len(vals)}


def main(workload, fetch_dir, write_dir, out=None):
    f = dominant(per_dispatch(fetch_dir, "FETCH_SIZE"))
    w = dominant(per_dispatch(write_dir, "WRITE_SIZE"))
    if f is None or w is None:
        print("no FIR dispatches found", file=sys.stderr)
        return 1
    fetch_bytes = f["mean_kib"] * 1024.0
    write_bytes = w["mean_kib"] * 1024.0
    res = {
        "kernel": f["kernel"], "grid_threads": f["grid_threads"], "launches": f["launches"],
        "fetch_size_raw_bytes": fetch_bytes, "write_size_bytes": write_bytes,
        "hbm_bytes_per_launch": 2.0 * fetch_bytes + write_bytes,
        "note": "traffic = 2 x FETCH_SIZE (gfx950 wide-read correction) + WRITE_SIZE, per launch",
    }
    data = {}
    if out and os.path.exists(out):
        with open(out) as fh:
            data = json.load(fh)
    data[workload] = res
    text = json.dumps(data, indent=1)
    if out:
        with open(out, "w") as fh:
            fh.write(text + "\n")
    print(text)
    return 0


if __name__ == "__main__":
    sys.exit(main(*sys.argv[1:]))
