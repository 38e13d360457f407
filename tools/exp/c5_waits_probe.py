#!/usr/bin/env python3
"""Hand-off wait profile of the fused C5 launch (firI8WsKernel<11, 3, AM, true>) on the GSDR_WS_WAITS
diagnostic build (GSDR_LIB=cuda-sdr_amd/lib_waits/...): after ~1 s of back-to-back bench-shaped C5
steps, one more step with the counters reset; per role (8 consumer waves, 4 producer waves per
workgroup) the share of each wave's span spent waiting on each hand-off counter."""
import ctypes
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "cuda-sdr_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from gpusdr import ops  # noqa: E402
from gpusdr._native import lib  # noqa: E402

KINDS = ["planesFull", "planesFree", "partsFull", "partsFree", "pstat", "tapsRead", "amSlot", "amFree"]
SLOTS = 13


def waits(reset):
    n = 256 * 12 * SLOTS
    buf = (ctypes.c_ulonglong * n)()
    assert lib().gsdrAmdWsWaits(buf, ctypes.c_size_t(n), int(reset)) == 0
    return np.frombuffer(buf, dtype=np.uint64).reshape(256, 12, SLOTS).astype(np.float64)


if __name__ == "__main__":
    dev = torch.device("cuda", 0)
    ws8 = "--ws8" in sys.argv  # the r04 8-way kernel (GSDR_POLICY_I8_WS8); default: the r05 4-way kernel
    if ws8:
        ops.set_kernel_policy(ops.POLICY_I8_WS8)
    nc = 8 if ws8 else 4  # consumer waves per workgroup; the producers follow (4)
    chain = bench.AmChainSharded(ops, 0, 1, dev)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 1.0:
        for _ in range(8):
            chain.step()
        torch.cuda.synchronize()
    waits(True)
    chain.step()
    torch.cuda.synchronize()
    w = waits(True)
    print(f"kernel: {'8-way (firI8WsKernel)' if ws8 else '4-way (firI8Ws4Kernel)'}")
    for role, sl in ((f"consumers (waves 0-{nc - 1})", slice(0, nc)), (f"producers (waves {nc}-{nc + 3})", slice(nc, nc + 4))):
        x = w[:, sl, :]
        span = x[..., 8].sum()
        parts = ", ".join(f"{k} {x[..., i].sum() / span * 100:.1f}%" for i, k in enumerate(KINDS) if x[..., i].sum() > 0)
        print(f"{role}: median span {np.median(x[..., 8]):.0f} cycles, waits {x[..., 9].sum() / x[..., 9].size:.0f} "
              f"per wave; share of span waiting: {parts}; total {x[..., :8].sum() / span * 100:.1f}%", flush=True)
        if not ws8 and sl.start == nc:  # the 4-way producers' phases (stamps)
            print("  producer phases (share of span): " + ", ".join(
                f"{k} {x[..., i].sum() / span * 100:.1f}%" for i, k in
                ((10, "audio stage"), (11, "window vmcnt wait"), (12, "planesFree wait"), (9, "convert+writes+load issue"))),
                flush=True)
        if not ws8 and sl.start == 0:  # the 4-way consumers' phases (stamps)
            print("  consumer phases (share of span): " + ", ".join(
                f"{k} {x[..., i].sum() / span * 100:.1f}%" for i, k in
                ((10, "MFMA loop"), (11, "partials write"), (12, "reduce+epilogue incl. its waits"))), flush=True)
    per_w = w[..., :8].sum(axis=2) / np.maximum(w[..., 8], 1)
    print("wait share by wave index (median over workgroups): " +
          " ".join(f"w{i}:{np.median(per_w[:, i]) * 100:.0f}%" for i in range(nc + 4)))
