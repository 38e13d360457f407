#!/usr/bin/env python3
"""bench.py's C3 step loop dissected: the FIR launch time (HIP events) under the exact bench loop,
without the per-step halo copy, and with one event pair around all steps."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "cuda-sdr_amd"))
sys.path.insert(0, REPO)
from gpusdr import ops  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda", 0)
chain = bench.ShardedChain(ops, "c3", 0, 1, dev)
sl = chain.slot
g = chain.geom


def run(mode, steps=20):
    torch.cuda.synchronize()
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    a.record()
    for i in range(steps):
        if mode == "bench":
            chain.step(evs[i])
        elif mode == "nocopy":
            evs[i][0].record()
            ops.fir(chain.taps, sl.buf, chain.D, g.outputs, out=sl.out, am=True)
            evs[i][1].record()
        elif mode == "noevents":
            ops.fir(chain.taps, sl.buf, chain.D, g.outputs, out=sl.out, am=True)
            sl.ring.halo.copy_(sl.ring.tail)
        elif mode == "plain":
            ops.fir(chain.taps, sl.buf, chain.D, g.outputs, out=sl.out, am=True)
    b.record()
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps * 1e3
    per = a.elapsed_time(b) / steps
    ev = np.mean([x.elapsed_time(y) for x, y in evs]) if mode in ("bench", "nocopy") else float("nan")
    return wall, per, ev


for rnd in range(3):
    for mode in ("bench", "nocopy", "noevents", "plain"):
        w, p, e = run(mode)
        print(f"round {rnd} {mode:9s} wall/step {w:6.3f} ms  events/step {p:6.3f} ms  per-launch events {e:6.3f} ms",
              flush=True)
