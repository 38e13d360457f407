#!/usr/bin/env python3
"""Why does the C3 FFT kernel take ~0.58 ms under bench.py but ~0.49 ms in tools/exp/fft_bench?
Times the same gsdrFirFCAmDemod launch (2^28 - 6 cf32, 1023 taps, D = 10) over inputs from
different allocators / streams / data, HIP events around 10 launches, interleaved rounds."""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(REPO, "cuda-sdr_amd"))
sys.path.insert(0, REPO)
from gpusdr import ops  # noqa: E402
from gpusdr._native import lib  # noqa: E402
import bench  # noqa: E402

L = lib()
hip = ctypes.CDLL("libamdhip64.so")
n_in = (1 << 28) - (1 << 28) % 10 + 1022
T, D = 1023, 10
n_out = (n_in - T) // D + 1
taps = torch.from_numpy(bench.lowpass(T, 0.04, "blackman")).cuda()
L.gsdrFirFCAmDemod.argtypes = [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p,
                               ctypes.c_size_t, ctypes.c_int32, ctypes.c_void_p]
L.gsdrFirFCAmDemod.restype = ctypes.c_int


def hip_malloc(nbytes):
    p = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(p), ctypes.c_size_t(nbytes)) == 0
    return p.value


cases = {}
xt = torch.empty(n_in, dtype=torch.complex64, device="cuda")
ops.synth_wideband_cf32(0xC3, 0.013, 0.31, 0, n_in, out=xt)
ot = torch.empty(n_out, dtype=torch.float32, device="cuda")
cases["torch alloc, torch stream"] = (xt.data_ptr(), ot.data_ptr(), torch.cuda.current_stream().cuda_stream)
xh = hip_malloc(n_in * 8)
oh = hip_malloc(n_out * 4)
hip.hipMemcpy(ctypes.c_void_p(xh), ctypes.c_void_p(xt.data_ptr()), ctypes.c_size_t(n_in * 8), 3)
cases["hipMalloc, torch stream"] = (xh, oh, torch.cuda.current_stream().cuda_stream)
cases["hipMalloc, null stream"] = (xh, oh, None)
s2 = torch.cuda.Stream()
cases["torch alloc, side stream"] = (xt.data_ptr(), ot.data_ptr(), s2.cuda_stream)
torch.cuda.synchronize()
res = {k: [] for k in cases}
for rnd in range(5):
    for name, (x, o, st) in cases.items():
        stream = torch.cuda.ExternalStream(st) if st else torch.cuda.default_stream()
        with torch.cuda.stream(stream):
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            for _ in range(2):
                assert L.gsdrFirFCAmDemod(D, taps.data_ptr(), T, x, o, n_out, 0, st) == 0
            a.record(stream)
            for _ in range(10):
                L.gsdrFirFCAmDemod(D, taps.data_ptr(), T, x, o, n_out, 0, st)
            b.record(stream)
            b.synchronize()
            res[name].append(a.elapsed_time(b) / 10)
for name, v in res.items():
    print(f"{name:32s} median {np.median(v) * 1e3:7.1f} us  min {np.min(v) * 1e3:7.1f} us", flush=True)
