#!/usr/bin/env python3
"""C5 RF stage (int8 IQ, 125 M samples + 3 600 halo, 1023 taps, D = 10, AM) on the wave-specialised
f16 MFMA kernel (default policy) vs the polyphase FFT kernel (GSDR_POLICY_PREFER_FFT): HIP events
around 10 launches each, interleaved rounds after a settle; max relative difference of the outputs."""
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

T, D = 1023, 10
L = 125_000_000 + 3600
n_out = (L - T) // D + 1
taps = torch.from_numpy(bench.lowpass(T, 0.04, "blackman")).cuda()
xs = [torch.empty(2 * L, dtype=torch.int8, device="cuda") for _ in range(4)]
for k, x in enumerate(xs):
    ops.synth_iq_int8(0x5EED, 1e9, 1e3, 1e9 * 0.075, k * L, L, out=x)
outs = {p: torch.empty(n_out, dtype=torch.float32, device="cuda") for p in ("mfma", "fft")}
pol = {"mfma": 0, "fft": ops.POLICY_PREFER_FFT}


def launch(p, x):
    ops.set_kernel_policy(pol[p])
    ops.fir(taps, x, D, n_out, out=outs[p], am=True, int8_iq=True)


for p in pol:
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:
        for x in xs:
            launch(p, x)
        torch.cuda.synchronize()
    print(p, "class", ops.fir_kernel_class(xs[0], taps, D, int8_iq=True), flush=True)
ts = {p: [] for p in pol}
for rnd in range(4):
    for p in pol:
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(12):
            launch(p, xs[i % 4])
        b.record()
        b.synchronize()
        ts[p].append(a.elapsed_time(b) / 12 * 1e3)
for p in pol:
    print(f"{p:5s} us/launch rounds {[round(v, 1) for v in ts[p]]} median {np.median(ts[p]):.1f}", flush=True)
launch("mfma", xs[0])
launch("fft", xs[0])
torch.cuda.synchronize()
a, b = outs["mfma"].double(), outs["fft"].double()
print("max |mfma - fft| / max|y|:", float((a - b).abs().max() / a.abs().max()))
print("direct blocks (fft):", ops.fft_direct_blocks(0, reset=True))
ops.set_kernel_policy(0)
