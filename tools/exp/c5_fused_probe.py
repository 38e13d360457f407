#!/usr/bin/env python3
"""C5 shape (125 M int8 IQ + 3 600 halo, RF 1023 taps D = 10, audio 255 taps D = 20): the fused
gsdrInt8FirFCAmDemodFirFF with the AM store on / off and with / without AM history, against the two
calls (gsdrInt8FirFCAmDemod + gsdrFirFF); HIP events around 10 launches each, interleaved rounds."""
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

T, D, Ta, Da = 1023, 10, 255, 20
L = 125_000_000 + 3600
n_rf = (L - T) // D + 1
rf = torch.from_numpy(bench.lowpass(T, 0.04, "blackman")).cuda()
au = torch.from_numpy(bench.lowpass(Ta, 0.02, "hamming")).cuda()
xs = [torch.empty(2 * L, dtype=torch.int8, device="cuda") for _ in range(3)]
for k, x in enumerate(xs):
    ops.synth_iq_int8(0x5EED, 1e9, 1e3, 1e9 * 0.075, k * L, L, out=x)
H = 257
am = torch.zeros(H + n_rf, dtype=torch.float32, device="cuda")
n_a0 = (n_rf - Ta) // Da + 1
n_aH = (H + n_rf - Ta) // Da + 1
out = torch.empty(max(n_a0, n_aH), dtype=torch.float32, device="cuda")


def two_calls(x):
    ops.fir(rf, x, D, n_rf, out=am[:n_rf], am=True, int8_iq=True)
    ops.fir(au, am[:n_rf], Da, n_a0, out=out[:n_a0])


cases = {
    "two calls": two_calls,
    "fused store=0 H=0": lambda x: ops.am_chain_fused(rf, x, D, n_rf, am, 0, au, Da, n_a0, out, store_am=False),
    "fused store=1 H=0": lambda x: ops.am_chain_fused(rf, x, D, n_rf, am, 0, au, Da, n_a0, out, store_am=True),
    "fused store=1 H=257": lambda x: ops.am_chain_fused(rf, x, D, n_rf, am, H, au, Da, n_aH, out, store_am=True),
    "fused store=0 H=257": lambda x: ops.am_chain_fused(rf, x, D, n_rf, am, H, au, Da, n_aH, out, store_am=False),
}
for name, f in cases.items():
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.25:
        for x in xs:
            f(x)
        torch.cuda.synchronize()
ts = {name: [] for name in cases}
for rnd in range(4):
    for name, f in cases.items():
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for i in range(9):
            f(xs[i % 3])
        b.record()
        b.synchronize()
        ts[name].append(a.elapsed_time(b) / 9 * 1e3)
for name in cases:
    print(f"{name:22s} us/step rounds {[round(v, 1) for v in ts[name]]} median {np.median(ts[name]):.1f}", flush=True)
print("ws aborts:", ops.ws_aborts(reset=True))
