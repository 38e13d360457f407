"""Does recording a HIP event pair around every step's launch (bench.py's live kernel timing) cost
wall time per step? C2 (36 us launches) and C3 (0.48 ms) stepped K times with and without the
per-step events, interleaved; per-step wall time and the event-measured launch time."""
import os
import sys
import time

import numpy as np
import torch

sys.path[:0] = [os.path.join(os.path.dirname(__file__), "..", ".."), os.path.join(os.path.dirname(__file__), "..", "..", "cuda-sdr_amd")]
import bench  # noqa: E402
from gpusdr import ops  # noqa: E402

dev = torch.device("cuda", 0)
for wl, K in (("c2", 400), ("c3", 40)):
    ch = bench.ShardedChain(ops, wl, 0, 1, dev)
    bench.settle(ch.step)
    res = {"events": [], "none": []}
    for rnd in range(3):
        for mode in ("events", "none"):
            evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(K)]
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(K):
                ch.step(evs[i] if mode == "events" else None)
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / K * 1e6
            kern = float(np.mean([a.elapsed_time(b) for a, b in evs])) * 1e3 if mode == "events" else float("nan")
            res[mode].append((dt, kern))
    for mode, v in res.items():
        print(f"{wl} {mode:6s} wall us/step " + " ".join(f"{d:7.1f}" for d, _ in v) +
              ("   event us/launch " + " ".join(f"{k:7.1f}" for _, k in v) if mode == "events" else ""), flush=True)
