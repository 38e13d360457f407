#!/usr/bin/env python3
"""r06: the cf32 MFMA kernels' guard on adversarial inputs, per kernel variant (WS f16, sync f16, bf16 x 3):
failing outputs / tiles against float64 for sparse impulses (T = 200, D = 3) and the non-finite leak
(T = 1023, D = 10). Diagnostic for tests/test_mfma_guard.py."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "oracle"), REPO, os.path.join(REPO, "cuda-sdr_amd")]
import oracle  # noqa: E402  (checker only)
from gpusdr import ops  # noqa: E402

oracle.lib()
POL = {"ws": ops.POLICY_NO_FFT, "sync": ops.POLICY_NO_FFT | ops.POLICY_NO_WS,
       "bf16": ops.POLICY_NO_FFT | ops.POLICY_CF_BF16}


def run(taps, x, D, n_out, pol):
    prev = ops.set_kernel_policy(pol)
    try:
        y = ops.fir(torch.from_numpy(taps).cuda(), torch.from_numpy(x).cuda(), D, n_out)
        torch.cuda.synchronize()
    finally:
        ops.set_kernel_policy(prev)
    return y.cpu().numpy()


def impulses(T, D, n_out=40_000):
    n_in = (n_out - 1) * D + T
    x = np.zeros(n_in, np.complex64)
    x[::997] = 1 + 1j
    taps = oracle.lowpass_taps(T, 0.4 / D, "blackman")
    y64, bound = oracle.fir_f64(taps, x, D, n_out)
    print(f"impulses T={T} D={D}: taps[0]={taps[0]:.3e} taps[-1]={taps[-1]:.3e} min|h|={np.abs(taps).min():.3e}")
    for name, pol in POL.items():
        y = run(taps, x, D, n_out, pol)
        err = np.abs(y.astype(np.complex128) - y64)
        bad = np.nonzero(~(err <= 1e-6 * bound + 1e-30))[0]
        print(f"  {name}: {bad.size} bad, tiles {sorted(set((bad // 512).tolist()))[:20]}",
              [(int(k), complex(y[k]), complex(y64[k])) for k in bad[:3]], flush=True)


def nonfinite():
    T, D, n_out = 1023, 10, 20000
    n_in = (n_out - 1) * D + T
    x = oracle.synth_wideband_cf32(7, 0.013, 0.31, 0, n_in)
    x[50_000] = np.inf
    x[120_003] = np.nan
    print("nan bits", hex(x.view(np.uint32)[2 * 120_003]), hex(x.view(np.uint32)[2 * 120_003 + 1]))
    taps = oracle.lowpass_taps(T, 0.04, "blackman")
    k = np.arange(n_out)
    touched = np.zeros(n_out, bool)
    for pos in (50_000, 120_003):
        touched |= (k * D <= pos) & (pos < k * D + T)
    for name, pol in POL.items():
        y = run(taps, x, D, n_out, pol)
        leaked = np.nonzero(~np.isfinite(y) & ~touched)[0]
        nf = np.nonzero(~np.isfinite(y))[0]
        print(f"  nonfinite {name}: leaked {leaked.size} tiles {sorted(set((leaked // 512).tolist()))}, "
              f"non-finite {nf.size} in [{nf.min() if nf.size else -1}, {nf.max() if nf.size else -1}]", flush=True)


impulses(200, 3)
impulses(1023, 10)
nonfinite()
