#!/usr/bin/env python3
"""the host-fed C5 leg of bench.py (gsdrAmChainStepHost: pinned hipHostMalloc input
slots, H2D on the chain's copy stream, the fused chain graph, audio D2H into pinned output slots) run
alone, so a rocprofv3 --kernel-trace --memory-copy-trace of this process shows where a chunk's time goes:
copy sizes / engines / durations against the kernel launches, and the gaps between them. Then the
chunk's H2D copy alone (pinned host -> device, 10 MB) at destination offsets 0, 2 060 (the staging
window's offset behind the RF history: 2 r bytes) and 4 096, the suspect being the misaligned destination."""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "cuda-sdr_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def h2d_rate(dev, nbytes, dst_off, src_off=0, reps=20):
    hb = torch.empty(nbytes + 8192, dtype=torch.int8, pin_memory=True)
    db = torch.empty(nbytes + 8192, dtype=torch.int8, device=dev)
    s = torch.cuda.Stream(dev)
    src, dst = hb[src_off: src_off + nbytes], db[dst_off: dst_off + nbytes]
    with torch.cuda.stream(s):
        for _ in range(3):
            dst.copy_(src, non_blocking=True)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(s)
        for _ in range(reps):
            dst.copy_(src, non_blocking=True)
        b.record(s)
    b.synchronize()
    return reps * nbytes / (a.elapsed_time(b) * 1e-3) / 1e9


def timed_loop(dev, slots=4, warmup=8, steps=48):
    """bench.host_fed_c5's loop with each host call timed (perf_counter): where a step's host time goes."""
    from gpusdr import ops
    from gpusdr.chain import AmChain
    desc, kind, L, T, D, cutoff, window, fs = bench.WORKLOADS["c5"]
    Ta, Da, cut_a, win_a = bench.C5_AUDIO
    chain = AmChain(bench.lowpass(T, cutoff, window), D, bench.lowpass(Ta, cut_a, win_a), Da, bench.C5_CHUNK,
                    dev.index, host_slots=slots)
    for s in range(slots):
        chain.host_input(s)[:] = ops.synth_iq_int8(0x5EED, fs, 1e3, fs * 0.075, s * bench.C5_CHUNK, bench.C5_CHUNK,
                                                   device=dev).cpu().numpy()
    counts = [0] * slots
    tw, ts = [], []
    t_start = time.perf_counter()
    for k in range(warmup + steps):
        s = k % slots
        if k >= slots:
            t0 = time.perf_counter()
            chain.wait_host(s, counts[s])
            tw.append(time.perf_counter() - t0)
        t0 = time.perf_counter()
        counts[s] = chain.step_host(s)
        ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    total = time.perf_counter() - t_start
    chain.close()
    import numpy as np
    return {"slots": slots, "ms_per_step": total / (warmup + steps) * 1e3,
            "wait_host_ms": {"median": float(np.median(tw)) * 1e3, "max": float(np.max(tw)) * 1e3,
                             "sum": float(np.sum(tw)) * 1e3},
            "step_host_ms": {"median": float(np.median(ts)) * 1e3, "max": float(np.max(ts)) * 1e3,
                             "sum": float(np.sum(ts)) * 1e3},
            "step_host_ms_each": [round(x * 1e3, 3) for x in ts[:24]],
            "wait_host_ms_each": [round(x * 1e3, 3) for x in tw[:24]]}


if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for slots in (4, 8):
        print(json.dumps(timed_loop(dev, slots)), flush=True)
    for slots in (4, 8):
        t0 = time.perf_counter()
        print(json.dumps(bench.host_fed_c5(dev, slots=slots)), flush=True)
    n = 2 * bench.C5_CHUNK
    for dst_off, src_off in ((0, 0), (2060, 0), (4096, 0), (2060, 2060)):
        print(json.dumps({"h2d_bytes": n, "dst_offset": dst_off, "src_offset": src_off,
                          "gbs": h2d_rate(dev, n, dst_off, src_off)}), flush=True)
