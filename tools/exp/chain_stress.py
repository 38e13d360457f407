#!/usr/bin/env python3
"""Repeat test_am_chain_device_steps' cases (the executor's per-step fused launches against the
float64 oracle) many times in one process, printing the failing indices of any run - r04 saw the
two short-filter cases fail once in a full suite run (profiles/r04/final/gpu_tests_full_u_2failed.log)."""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "cuda-sdr_amd"), os.path.join(REPO, "oracle"), os.path.join(REPO, "tests")]
import oracle as orc  # noqa: E402
from gpusdr import chain as chain_mod  # noqa: E402
from test_am_chain import _expected  # noqa: E402

CASES = [(127, 1, 63, 4, 2048), (64, 3, 31, 5, 3000), (1023, 10, 255, 20, 4000)]
reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
fails = 0
for rep in range(reps):
    for T, D, Ta, Da, L in CASES:
        rng = np.random.default_rng(T + L + 7919 * rep)
        rf = orc.lowpass_taps(T, 0.4 / D)
        au = orc.lowpass_taps(Ta, 0.4 / Da)
        c = chain_mod.AmChain(rf, D, au, Da, L)
        steps = 7
        iq = rng.integers(-128, 128, size=2 * L * steps).astype(np.int8)
        dev = torch.from_numpy(iq).cuda()
        outs = [c.step(dev[2 * L * s: 2 * L * (s + 1)]).cpu().numpy() for s in range(steps)]
        got = np.concatenate(outs)
        want, bound = _expected(orc, iq, rf, D, au, Da)
        bad = np.nonzero(~(np.abs(got - want) <= bound))[0]
        if bad.size:
            fails += 1
            n0 = len(outs[0])
            print(f"rep {rep} case {(T, D, Ta, Da, L)}: {bad.size} of {len(got)} bad; idx {bad[:16].tolist()}; "
                  f"steps {((bad[:16] - n0) // max(1, L // (D * Da)) + 1).tolist()}; got {got[bad[:4]]} want {want[bad[:4]]}",
                  flush=True)
        c.close()
    print(f"rep {rep} done, failures so far {fails}", flush=True)
print("stress done, failures", fails)
