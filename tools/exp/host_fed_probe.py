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


if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    for slots in (4, 8):
        t0 = time.perf_counter()
        print(json.dumps(bench.host_fed_c5(dev, slots=slots)), flush=True)
    n = 2 * bench.C5_CHUNK
    for dst_off, src_off in ((0, 0), (2060, 0), (4096, 0), (2060, 2060)):
        print(json.dumps({"h2d_bytes": n, "dst_offset": dst_off, "src_offset": src_off,
                          "gbs": h2d_rate(dev, n, dst_off, src_off)}), flush=True)
