#!/usr/bin/env python3
"""does the complex-output FFT launch plus a separate gsdrQuadAmDemod beat the
AM-epilogue launch (gsdrFirFCAmDemod) at the C3 shape? HIP events around `reps` launches per arm,
arms interleaved over rounds, input slots rotating past the 256 MB Infinity Cache (as bench.py).
Arms: am (the headline launch), cplx (gsdrFirFC only), cplx+am (gsdrFirFC then gsdrQuadAmDemod),
amk (gsdrQuadAmDemod alone over the cf32 intermediate). Run under rocprofv3 --kernel-trace --stats
to see the kernels (r04: under rocprofv3 --kernel-trace)."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "cuda-sdr_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from gpusdr import ops  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    desc, kind, L, T, D, cutoff, window, fs = bench.WORKLOADS["c3"]
    n_out = (L - T) // D + 1
    n_in = (n_out - 1) * D + T
    taps = torch.from_numpy(bench.lowpass(T, cutoff, window)).to(dev)
    slots = []
    for k in range(3):
        x = torch.empty(n_in, dtype=torch.complex64, device=dev)
        ops.synth_wideband_cf32(0xC3, 0.013, 0.31, k * L, n_in, out=x)
        slots.append(x)
    out_am = torch.empty(n_out, dtype=torch.float32, device=dev)
    out_c = [torch.empty(n_out, dtype=torch.complex64, device=dev) for _ in range(2)]
    torch.cuda.synchronize()

    def arm_am(i):
        ops.fir(taps, slots[i % 3], D, n_out, out=out_am, am=True)

    def arm_cplx(i):
        ops.fir(taps, slots[i % 3], D, n_out, out=out_c[i % 2])

    def arm_cplx_am(i):
        ops.fir(taps, slots[i % 3], D, n_out, out=out_c[i % 2])
        ops.quad_am_demod(out_c[i % 2], out=out_am)

    def arm_amk(i):
        ops.quad_am_demod(out_c[i % 2], out=out_am)

    arms = {"am": arm_am, "cplx": arm_cplx, "cplx+am": arm_cplx_am, "amk": arm_amk}
    # settle: ~0.5 s of the headline launch
    t0 = time.perf_counter()
    i = 0
    while time.perf_counter() - t0 < 0.5:
        arm_am(i)
        i += 1
        if i % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    reps = int(os.environ.get("REPS", "20"))
    res = {k: [] for k in arms}
    for rd in range(int(os.environ.get("ROUNDS", "6"))):
        for name, fn in arms.items():
            for w in range(3):
                fn(w)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for r in range(reps):
                fn(r)
            b.record()
            b.synchronize()
            res[name].append(a.elapsed_time(b) / reps * 1e3)
    alg = n_in * 8 + n_out * 4
    for name, ts in res.items():
        med = float(np.median(ts))
        print(f"{name:8s} median {med:8.1f} us  min {min(ts):8.1f} us  "
              f"({alg / (med * 1e-6) / 1e12:.3f} TB/s of the AM chain's algorithmic bytes)", flush=True)
    print(f"n_out {n_out}, n_in {n_in}, kernel class {ops.fir_kernel_class(slots[0], taps, D)}")


if __name__ == "__main__":
    main()
