"""CPU oracle for the FIR -> QuadAmDemod hot path.  TEST INFRASTRUCTURE ONLY.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module: it is the checker and the timed CPU baseline, never the product path.

Two layers:

* ``liborcl.so`` (oracle/gsdr_oracle.c): the arithmetic - float64 FIR reference with the
  parity-tolerance scale, the exact int8 / AM expressions, phase cosines, the synthetic
  sources and the multithreaded float32 CPU baseline.  Reference lines are cited there.
* ``FirStreamModel`` / ``ElementwiseStreamModel`` below: a restatement of the reference's
  streaming contract - the BaseSink input window (src/filters/BaseSink.cpp:61-170), the
  FIR count / consume rule (src/filters/Fir.cpp:141-197, :210-279) and partial reads into
  a small output buffer (tests/FirTests.cpp:96-221) - so chunked GPU runs can be replayed
  on the CPU step by step.

Pinning: tests/test_oracle_golden.py checks this oracle against the reference's FIR and
cosine known-answer tests (tests/FirTests.cpp, tests/CosineSourceTests.cpp) and against
independent numpy float64 fixtures in tests/golden/.
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "_build", "liborcl.so")
_LIB_V4_PATH = os.path.join(_HERE, "_build", "liborcl_v4.so")
_lib = None
_baseline_lib = None

SAMPLE_FLOAT_COMPLEX = 0  # SampleType.h:20-25
SAMPLE_FLOAT = 1
SAMPLE_INT8_COMPLEX = 2


def build() -> str:
    """Compile liborcl.so with oracle/Makefile (gcc only; no GPU toolchain needed)."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def host_has_avx512() -> bool:
    """x86-64-v4 needs avx512f/bw/dq/vl (the flags gcc's -march=x86-64-v4 assumes)."""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("flags"):
                    flags = set(line.split(":", 1)[1].split())
                    return {"avx512f", "avx512bw", "avx512dq", "avx512vl"} <= flags
    except OSError:
        pass
    return False


def baseline_isa() -> str:
    return "x86-64-v4 (AVX-512)" if host_has_avx512() and os.path.exists(_LIB_V4_PATH) else "x86-64-v3 (AVX2+FMA)"


def baseline_lib():
    """The timed CPU baseline's library: the AVX-512 build when the host supports it."""
    global _baseline_lib
    if _baseline_lib is None:
        if host_has_avx512() and os.path.exists(_LIB_V4_PATH):
            _baseline_lib = _declare(ctypes.CDLL(_LIB_V4_PATH))
        else:
            _baseline_lib = lib()
    return _baseline_lib


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = _declare(ctypes.CDLL(_LIB_PATH))
    return _lib


def _declare(L):
    sz, vp, f32, f64, i32, u64 = (ctypes.c_size_t, ctypes.c_void_p, ctypes.c_float, ctypes.c_double,
                                  ctypes.c_int, ctypes.c_uint64)
    L.orc_fir_output_count.argtypes = [sz, sz, sz]
    L.orc_fir_output_count.restype = sz
    L.orc_fir_f64.argtypes = [i32, i32, sz, vp, sz, vp, vp, vp, sz]
    L.orc_int8_to_norm.argtypes = [ctypes.c_int8]
    L.orc_int8_to_norm.restype = f32
    L.orc_int8_to_float.argtypes = [vp, vp, sz]
    L.orc_quad_am_demod.argtypes = [vp, vp, sz]
    L.orc_multiply_cc.argtypes = [vp, vp, vp, sz]
    L.orc_quad_fm_demod_f64.argtypes = [vp, f64, vp, sz]
    L.orc_cosine_f.argtypes = [f32, f32, vp, sz]
    L.orc_cosine_c.argtypes = [f32, f32, vp, sz]
    L.orc_synth_iq_int8.argtypes = [u64, f64, f64, f64, u64, vp, sz]
    L.orc_synth_wideband_cf32.argtypes = [u64, f64, f64, u64, vp, sz]
    L.orc_chain_i8_fc_am_f32.argtypes = [sz, vp, sz, vp, vp, sz, i32]
    L.orc_chain_fc_am_f32.argtypes = [sz, vp, sz, vp, vp, sz, i32]
    L.orc_fir_ff_f32.argtypes = [sz, vp, sz, vp, vp, sz, i32]
    return L


def _ptr(a: np.ndarray) -> int:
    assert a.flags["C_CONTIGUOUS"]
    return a.ctypes.data


# ---- arithmetic -------------------------------------------------------------------------------

def fir_output_count(num_inputs: int, tap_count: int, decimation: int) -> int:
    return int(lib().orc_fir_output_count(num_inputs, tap_count, decimation))


def fir_f64(taps: np.ndarray, x: np.ndarray, decimation: int, n_out: int | None = None):
    """Float64 y[k] = sum_j h[j] x[kD+j] and the tolerance scale sum_j |h_j||x_kD+j|.

    ``taps``: float32 (real) or complex64; ``x``: float32 (real) or complex64.
    Returns (y complex128 or float64, bound float64)."""
    taps_c = np.iscomplexobj(taps)
    x_c = np.iscomplexobj(x)
    t = np.ascontiguousarray(taps, dtype=np.complex64 if taps_c else np.float32)
    xx = np.ascontiguousarray(x, dtype=np.complex64 if x_c else np.float32)
    D = max(1, int(decimation))
    T = len(t)
    if n_out is None:
        n_out = fir_output_count(len(xx), T, D)
    if n_out > 0:
        assert (n_out - 1) * D + T <= len(xx), "not enough input for n_out"
    out = np.zeros(2 * max(n_out, 1), dtype=np.float64)
    bound = np.zeros(max(n_out, 1), dtype=np.float64)
    lib().orc_fir_f64(int(taps_c), int(x_c), D, _ptr(t), T, _ptr(xx), _ptr(out), _ptr(bound), n_out)
    y = out[: 2 * n_out].view(np.complex128)
    if not taps_c and not x_c:
        y = y.real.copy()
    return y, bound[:n_out]


def int8_to_float(x: np.ndarray) -> np.ndarray:
    xx = np.ascontiguousarray(x, dtype=np.int8)
    out = np.empty(len(xx), dtype=np.float32)
    lib().orc_int8_to_float(_ptr(xx), _ptr(out), len(xx))
    return out


def quad_am_demod(z: np.ndarray) -> np.ndarray:
    zz = np.ascontiguousarray(z, dtype=np.complex64)
    out = np.empty(len(zz), dtype=np.float32)
    lib().orc_quad_am_demod(_ptr(zz), _ptr(out), len(zz))
    return out


def multiply_cc(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    """gsdrMultiplyCC restated (Multiply.cpp:145): non-conjugate product, bit-exact."""
    aa = np.ascontiguousarray(a, dtype=np.complex64)
    bb = np.ascontiguousarray(b, dtype=np.complex64)
    out = np.empty(max(len(aa), 1), dtype=np.complex64)
    lib().orc_multiply_cc(_ptr(aa), _ptr(bb), _ptr(out), len(aa))
    return out[: len(aa)]


def quad_fm_demod_f64(z: np.ndarray, gain: float) -> np.ndarray:
    """gsdrQuadFmDemod restated (QuadFmDemod.cpp:80-115): len(z) - 1 outputs; the float32
    product as the kernel forms it, atan2 in float64."""
    zz = np.ascontiguousarray(z, dtype=np.complex64)
    n = max(len(zz) - 1, 0)
    out = np.empty(max(n, 1), dtype=np.float64)
    lib().orc_quad_fm_demod_f64(_ptr(zz), float(gain), _ptr(out), n)
    return out[:n]


def mix_phase_fraction(rad: float) -> int:
    """Radians -> the 64-bit cycle fraction the fused mixer uses (include/gsdr/gsdr_amd.h)."""
    import math
    c = rad / 6.283185307179586476925286766559
    c -= math.floor(c)
    return int(math.ldexp(c, 64))


def mix_f64(x: np.ndarray, phase0: float, step: float) -> np.ndarray:
    """The fused frequency shifter restated: sample n times exp(j theta(n)), theta(n) the float32
    value of 2 pi (P0 + n F mod 2^64) / 2^64 (signed), the exponential in float64."""
    n = np.arange(len(x), dtype=np.uint64)
    ph = np.uint64(mix_phase_fraction(phase0)) + n * np.uint64(mix_phase_fraction(step))  # wraps mod 2^64
    th = (ph.view(np.int64).astype(np.float64) * 3.4061215800865545e-19).astype(np.float32)
    return np.asarray(x, dtype=np.complex128) * np.exp(1j * th.astype(np.float64))


def fm_gain(sample_rate: float, fsk_deviation: float) -> float:
    """QuadDemodFactory.h:111 (float arithmetic as in the reference)."""
    return float(np.float32(sample_rate) / (np.float32(2.0) * np.float32(np.pi) * np.float32(fsk_deviation) * np.float32(5)))


def cosine_f(phi_begin: float, phi_end: float, n: int) -> np.ndarray:
    out = np.empty(max(n, 1), dtype=np.float32)
    lib().orc_cosine_f(phi_begin, phi_end, _ptr(out), n)
    return out[:n]


def cosine_c(phi_begin: float, phi_end: float, n: int) -> np.ndarray:
    out = np.empty(max(n, 1), dtype=np.complex64)
    lib().orc_cosine_c(phi_begin, phi_end, _ptr(out), n)
    return out[:n]


def synth_iq_int8(seed: int, fs: float, am_hz: float, carrier_hz: float, first: int, n: int) -> np.ndarray:
    out = np.empty(2 * max(n, 1), dtype=np.int8)
    lib().orc_synth_iq_int8(seed, fs, am_hz, carrier_hz, first, _ptr(out), n)
    return out[: 2 * n]


def synth_wideband_cf32(seed: int, f1: float, f2: float, first: int, n: int) -> np.ndarray:
    out = np.empty(max(n, 1), dtype=np.complex64)
    lib().orc_synth_wideband_cf32(seed, f1, f2, first, _ptr(out), n)
    return out[:n]


def chain_i8_fc_am_f32(taps, iq, decimation, n_out, threads=1, baseline=False) -> np.ndarray:
    """CPU baseline: int8 IQ -> cf32 -> FC FIR -> AM envelope, float32 direct form."""
    t = np.ascontiguousarray(taps, dtype=np.float32)
    x = np.ascontiguousarray(iq, dtype=np.int8)
    out = np.empty(max(n_out, 1), dtype=np.float32)
    (baseline_lib() if baseline else lib()).orc_chain_i8_fc_am_f32(decimation, _ptr(t), len(t), _ptr(x), _ptr(out),
                                                                   n_out, threads)
    return out[:n_out]


def chain_fc_am_f32(taps, x, decimation, n_out, threads=1, baseline=False) -> np.ndarray:
    t = np.ascontiguousarray(taps, dtype=np.float32)
    xx = np.ascontiguousarray(x, dtype=np.complex64)
    out = np.empty(max(n_out, 1), dtype=np.float32)
    (baseline_lib() if baseline else lib()).orc_chain_fc_am_f32(decimation, _ptr(t), len(t), _ptr(xx), _ptr(out),
                                                                n_out, threads)
    return out[:n_out]


def fir_ff_f32(taps, x, decimation, n_out, threads=1, baseline=False) -> np.ndarray:
    """C1 CPU configuration: real f32 FIR, float32 direct form, `threads` time shards."""
    t = np.ascontiguousarray(taps, dtype=np.float32)
    xx = np.ascontiguousarray(x, dtype=np.float32)
    out = np.empty(max(n_out, 1), dtype=np.float32)
    (baseline_lib() if baseline else lib()).orc_fir_ff_f32(decimation, _ptr(t), len(t), _ptr(xx), _ptr(out), n_out,
                                                           threads)
    return out[:n_out]


# ---- streaming contract restatement -----------------------------------------------------------

class FirStreamModel:
    """The reference Fir filter's sink/source contract on the CPU, in float64.

    push(x)          ~ requestBuffer + copy + commitBuffer       (BaseSink.cpp:61-116)
    output_count()   ~ Fir::getNumOutputElements                 (Fir.cpp:141-186)
    read(max_out)    ~ Fir::readOutput into a buffer holding max_out elements:
                       n = min(available, max_out); consume n*D  (Fir.cpp:210-279)
    """

    def __init__(self, taps, decimation):
        self.taps = np.asarray(taps)
        self.D = max(1, int(decimation))
        self.complex_in = None
        self.buf = None

    def push(self, x):
        x = np.asarray(x)
        if self.buf is None:
            self.buf = x.copy()
        else:
            self.buf = np.concatenate([self.buf, x])

    def available_inputs(self) -> int:
        return 0 if self.buf is None else len(self.buf)

    def output_count(self) -> int:
        return fir_output_count(self.available_inputs(), len(self.taps), self.D)

    def read(self, max_out: int):
        n = min(self.output_count(), int(max_out))
        if n == 0:
            cplx = np.iscomplexobj(self.taps) or (self.buf is not None and np.iscomplexobj(self.buf))
            return np.zeros(0, dtype=np.complex128 if cplx else np.float64), np.zeros(0)
        y, bound = fir_f64(self.taps, self.buf, self.D, n)
        self.buf = self.buf[n * self.D:]
        return y, bound


class ElementwiseStreamModel:
    """QuadAmDemod / Int8ToFloat window contract: n = min(in_count, out_capacity), consume n
    input elements (QuadAmDemod.cpp:80-107, Int8ToFloat.cpp:80-100)."""

    def __init__(self, fn):
        self.fn = fn
        self.buf = None

    def push(self, x):
        x = np.asarray(x)
        self.buf = x.copy() if self.buf is None else np.concatenate([self.buf, x])

    def read(self, max_out: int):
        n = 0 if self.buf is None else min(len(self.buf), int(max_out))
        if n == 0:
            return self.fn(self.buf[:0] if self.buf is not None else np.zeros(0))
        y = self.fn(self.buf[:n])
        self.buf = self.buf[n:]
        return y


# ---- tap design (fixtures and bench; the reference's remez is absent) --------

def lowpass_taps(num_taps: int, cutoff: float, window: str = "hamming") -> np.ndarray:
    """Windowed-sinc low-pass designed in float64, unit DC gain, returned as float32.
    cutoff is in cycles/sample (0 < cutoff < 0.5)."""
    n = np.arange(num_taps, dtype=np.float64) - (num_taps - 1) / 2.0
    h = 2.0 * cutoff * np.sinc(2.0 * cutoff * n)
    if num_taps > 1:
        m = np.arange(num_taps, dtype=np.float64)
        if window == "hamming":
            w = 0.54 - 0.46 * np.cos(2.0 * np.pi * m / (num_taps - 1))
        elif window == "blackman":
            w = (0.42 - 0.5 * np.cos(2.0 * np.pi * m / (num_taps - 1))
                 + 0.08 * np.cos(4.0 * np.pi * m / (num_taps - 1)))
        else:
            raise ValueError(window)
        h = h * w
    h = h / h.sum()
    return h.astype(np.float32)
