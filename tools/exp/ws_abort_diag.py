#!/usr/bin/env python3
"""run the wave-specialised abort scenario of tests/test_am_chain.py
(test_am_chain_reports_ws_abort: resident chain steps with the spin limit at 0, every hand-off wait
returning early) and the fused sharded C5 step, on a diagnostic build of the library
(GSDR_LIB=cuda-sdr_amd/lib_diag/..., -DGSDR_WS_DIAG=1), then print the bounds-check counters of the
fused audio stage and the AM ring writes (gsdrAmdWsDiag): [0] aborted audio-tile waits, [1] history
index outside [0, amH), [2] AM index outside the ring tiles a window may span, [3] ring write outside
the ring, [4] history reads, [5] ring reads."""
import ctypes
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "cuda-sdr_amd"), os.path.join(REPO, "oracle")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import oracle as orc  # noqa: E402
from gpusdr import chain as chain_mod  # noqa: E402
from gpusdr import ops  # noqa: E402
from gpusdr._native import HipError, lib  # noqa: E402

NAMES = ["aborted_waits", "hist_oob", "ring_window_oob", "ring_write_oob", "hist_reads", "ring_reads", "audio_tiles",
         "audio_batches"]


def diag(reset=True):
    v = (ctypes.c_ulonglong * 8)()
    assert lib().gsdrAmdWsDiag(v, int(reset)) == 0
    return dict(zip(NAMES, list(v)))


def scenario(spin):
    T, D, Ta, Da, L = 1023, 10, 255, 20, 1_000_000
    rng = np.random.default_rng(19)
    rf = orc.lowpass_taps(T, 0.04)
    au = orc.lowpass_taps(Ta, 0.02)
    dev = torch.from_numpy(rng.integers(-128, 128, size=2 * L * 4).astype(np.int8)).cuda()
    ops.ws_aborts(reset=True)
    prev = ops.set_ws_spin_limit(spin)
    failed = 0
    try:
        c = chain_mod.AmChain(rf, D, au, Da, L)
        out = torch.empty(4 * (L // (D * Da)), dtype=torch.float32, device="cuda")
        # the test's sequence, within the resident API's contract (a non-first step reads its RF
        # history in place in front of its input, so it must be a later view of the same stream; after
        # a failed step the chain is reset and the next step is a first step again)
        for k in range(3):
            if k == 2:
                c.reset()  # step 2 starts the stream again at dev[0] (a first step) in every case
            try:
                c.step_resident(dev if k != 1 else dev[2 * L * 2:], 2, out)
            except HipError:
                failed += 1
            c.torch_stream.synchronize()
        aborts = ops.ws_aborts(reset=True)
        c.close()
    finally:
        ops.set_ws_spin_limit(prev)
        ops.ws_aborts(reset=True)
    return failed, aborts


def history_scenario(spin):
    """r05: a steady resident step - its audio windows reach into the AM history
    (amH > 0, the history branch) - under `spin`, after a first step at the normal limit."""
    T, D, Ta, Da, L = 1023, 10, 255, 20, 1_000_000
    rng = np.random.default_rng(23)
    rf = orc.lowpass_taps(T, 0.04)
    au = orc.lowpass_taps(Ta, 0.02)
    dev = torch.from_numpy(rng.integers(-128, 128, size=2 * L * 4).astype(np.int8)).cuda()
    ops.ws_aborts(reset=True)
    c = chain_mod.AmChain(rf, D, au, Da, L)
    out = torch.empty(4 * (L // (D * Da)), dtype=torch.float32, device="cuda")
    c.step_resident(dev, 2, out)  # first step, normal limit
    c.torch_stream.synchronize()
    diag(True)
    prev = ops.set_ws_spin_limit(spin)
    failed = 0
    try:
        try:
            c.step_resident(dev[2 * L * 2:], 2, out)  # steady: RF history in place, AM history amH > 0
        except HipError:
            failed += 1
        c.torch_stream.synchronize()
        aborts = ops.ws_aborts(reset=True)
        c.close()
    finally:
        ops.set_ws_spin_limit(prev)
        ops.ws_aborts(reset=True)
    return failed, aborts


if __name__ == "__main__":
    diag(True)
    # the same launches at the normal limit first: their batch count is the model for the aborted runs
    for spin in (1 << 22, 0, 0):
        failed, aborts = scenario(spin)
        print(f"spin limit {spin}: failed steps {failed}, abort count left {aborts}, diag {diag(True)}", flush=True)
    for spin in (1 << 22, 0, 0):
        failed, aborts = history_scenario(spin)
        print(f"steady step (amH > 0), spin limit {spin}: failed {failed}, aborts {aborts}, diag {diag(True)}",
              flush=True)
