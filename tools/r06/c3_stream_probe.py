#!/usr/bin/env python3
"""r06: C3 at the streaming granularity - where a 2^22-sample step's time goes.
(1) One launch of the C3 filter (1023 taps, D = 10, AM) over 2^22 - 4 samples on each kernel family: the FFT
kernel (default) and the wave-specialised f16 MFMA kernel (GSDR_POLICY_NO_FFT), HIP-event medians over
interleaved rounds, input rotated over 12 buffers (past the Infinity Cache). (2) bench.stream_path (the node
chain, push + replayed step) under each policy."""
import os
import sys
import time

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "cuda-sdr_amd")]
import bench  # noqa: E402
from gpusdr import ops  # noqa: E402

dev = torch.device("cuda", 0)
T, D = 1023, 10
taps = torch.from_numpy(bench.lowpass(T, 0.04, "blackman")).to(dev)
for n_in in ((1 << 22) - 4, 1 << 24, 1 << 26):
    n_out = (n_in - T) // D + 1
    xs = []
    for k in range(12):
        x = torch.empty(n_in, dtype=torch.complex64, device=dev)
        ops.synth_wideband_cf32(0xC3, 0.013, 0.31, k * n_in, n_in, out=x)
        xs.append(x)
    out = torch.empty(n_out, dtype=torch.float32, device=dev)
    res = {}
    for rnd in range(3):
        for name, pol in (("fft", 0), ("cf-mfma", ops.POLICY_NO_FFT)):
            prev = ops.set_kernel_policy(pol)
            try:
                for i in range(40):  # settle
                    ops.fir(taps, xs[i % 12], D, n_out, out=out, am=True)
                ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(48)]
                for i, (a, b) in enumerate(ev):
                    a.record()
                    ops.fir(taps, xs[i % 12], D, n_out, out=out, am=True)
                    b.record()
                torch.cuda.synchronize()
                res.setdefault(name, []).append(float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3)
                cls = ops.fir_kernel_class(xs[0], taps, D)
            finally:
                ops.set_kernel_policy(prev)
            res.setdefault(name + "_class", cls)
    print(f"n_in {n_in}: " + ", ".join(f"{k} {v if isinstance(v, str) else [round(t, 2) for t in v]}"
                                       for k, v in res.items()) + " us per launch", flush=True)
    del xs
    torch.cuda.empty_cache()

for name, pol in (("default", 0), ("no-fft", ops.POLICY_NO_FFT)):
    prev = ops.set_kernel_policy(pol)
    try:
        r = bench.stream_path(ops, dev, 552_000.0)
    finally:
        ops.set_kernel_policy(prev)
    print(name, {k: r[k] for k in ("value", "ms_per_step", "gpu_ms_per_step", "host_us_per_step")}, r["graph"],
          flush=True)
