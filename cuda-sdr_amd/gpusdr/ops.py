"""Tensor-level wrappers over the gsdr C-ABI (include/gsdr/*.h).

Plumbing only: torch provides device memory and the current HIP stream; every call goes
straight to a hand-written gfx950 kernel in libgpusdrpipeline.so. Each wrapper mirrors one
reference entry point (argument meaning and the FIR count rule of src/filters/Fir.cpp).
"""
from __future__ import annotations

import ctypes

import torch

from ._native import HipError, check, lib


def _stream(t: torch.Tensor):
    return torch.cuda.current_stream(t.device).cuda_stream


def _dev(t: torch.Tensor) -> int:
    return t.device.index if t.device.index is not None else torch.cuda.current_device()


def _require(t: torch.Tensor, dtype, name: str):
    if not t.is_cuda:
        raise ValueError(f"{name} must be a device tensor")
    if t.dtype != dtype:
        raise ValueError(f"{name} must be {dtype}, got {t.dtype}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")


def fir_output_count(num_inputs: int, tap_count: int, decimation: int) -> int:
    """Fir.cpp:178-186 with the size_t wrap guarded."""
    d = max(1, int(decimation))
    if tap_count == 0 or num_inputs < tap_count:
        return 0
    return (num_inputs - (tap_count - 1)) // d


_FIR_ENTRY = {
    # (taps complex, input kind, am epilogue) -> entry point
    (False, "f32", False): "gsdrFirFF",
    (False, "c64", False): "gsdrFirFC",
    (True, "c64", False): "gsdrFirCC",
    (True, "f32", False): "gsdrFirCF",
    (False, "c64", True): "gsdrFirFCAmDemod",
    (True, "c64", True): "gsdrFirCCAmDemod",
    (False, "i8iq", False): "gsdrInt8FirFC",
    (False, "i8iq", True): "gsdrInt8FirFCAmDemod",
}


_MIX_ENTRY = {("c64", False): "gsdrMixFirFC", ("c64", True): "gsdrMixFirFCAmDemod",
              ("i8iq", False): "gsdrInt8MixFirFC", ("i8iq", True): "gsdrInt8MixFirFCAmDemod"}


def fir(taps: torch.Tensor, x: torch.Tensor, decimation: int = 1, num_outputs: int | None = None,
        out: torch.Tensor | None = None, am: bool = False, int8_iq: bool = False,
        mix: tuple[float, float] | None = None) -> torch.Tensor:
    """y[k] = sum_j taps[j] * x[k*D + j] on the GPU.

    taps: float32 (real) or complex64, device.  x: float32, complex64, or (int8_iq=True) int8
    interleaved I/Q.  am=True fuses the QuadAmDemod envelope (float32 output).
    mix=(phase0, radians_per_sample): frequency-shift the (complex) input first, fused into the
    load (gsdr*MixFirFC*; real taps only)."""
    taps_c = taps.dtype == torch.complex64
    _require(taps, torch.complex64 if taps_c else torch.float32, "taps")
    if int8_iq:
        _require(x, torch.int8, "x")
        kind, n_in = "i8iq", x.numel() // 2
    elif x.dtype == torch.complex64:
        _require(x, torch.complex64, "x")
        kind, n_in = "c64", x.numel()
    else:
        _require(x, torch.float32, "x")
        kind, n_in = "f32", x.numel()
    key = (taps_c, kind, am)
    if key not in _FIR_ENTRY:
        raise ValueError(f"unsupported FIR combination {key}")
    d = max(1, int(decimation))
    T = taps.numel()
    if num_outputs is None:
        num_outputs = fir_output_count(n_in, T, d)
    if num_outputs > 0 and (num_outputs - 1) * d + T > n_in:
        raise ValueError("input too short for the requested outputs")
    out_dtype = torch.float32 if (am or (not taps_c and kind == "f32")) else torch.complex64
    if out is None:
        out = torch.empty(num_outputs, dtype=out_dtype, device=x.device)
    else:
        _require(out, out_dtype, "out")
        if out.numel() < num_outputs:
            raise ValueError("out too small")
    if num_outputs == 0:
        return out
    if mix is not None:
        if taps_c or kind == "f32":
            raise ValueError("mix needs real taps and complex input")
        fn = getattr(lib(), _MIX_ENTRY[(kind, am)])
        check(fn(d, taps.data_ptr(), T, x.data_ptr(), float(mix[0]), float(mix[1]), out.data_ptr(), num_outputs,
                 _dev(x), _stream(x)), fn.__name__)
        return out
    fn = getattr(lib(), _FIR_ENTRY[key])
    check(fn(d, taps.data_ptr(), T, x.data_ptr(), out.data_ptr(), num_outputs, _dev(x), _stream(x)), fn.__name__)
    return out


def bind_fir(taps: torch.Tensor, x: torch.Tensor, decimation: int, num_outputs: int, out: torch.Tensor,
             am: bool = False, int8_iq: bool = False):
    """The launch `fir(taps, x, decimation, num_outputs, out=out, am=am, int8_iq=int8_iq)` validated
    once and bound to fixed addresses and torch's current stream: returns a zero-argument callable
    that only enqueues the kernel (a few microseconds of host time instead of the argument checks -
    what a step loop over fixed buffers needs when the kernel itself takes tens of microseconds)."""
    taps_c = taps.dtype == torch.complex64
    _require(taps, torch.complex64 if taps_c else torch.float32, "taps")
    kind = "i8iq" if int8_iq else ("c64" if x.dtype == torch.complex64 else "f32")
    _require(x, {"i8iq": torch.int8, "c64": torch.complex64, "f32": torch.float32}[kind], "x")
    key = (taps_c, kind, am)
    if key not in _FIR_ENTRY:
        raise ValueError(f"unsupported FIR combination {key}")
    d, T = max(1, int(decimation)), taps.numel()
    n_in = x.numel() // 2 if int8_iq else x.numel()
    if num_outputs > 0 and (num_outputs - 1) * d + T > n_in:
        raise ValueError("input too short for the requested outputs")
    out_dtype = torch.float32 if (am or (not taps_c and kind == "f32")) else torch.complex64
    _require(out, out_dtype, "out")
    if out.numel() < num_outputs:
        raise ValueError("out too small")
    fn = getattr(lib(), _FIR_ENTRY[key])
    args = (d, taps.data_ptr(), T, x.data_ptr(), out.data_ptr(), int(num_outputs), _dev(x), _stream(x))
    name = fn.__name__
    keep = (taps, x, out)  # the bound addresses stay valid while the callable lives

    def launch():
        if num_outputs > 0:
            code = fn(*args)
            if code != 0:
                raise HipError(f"{name} failed with hipError_t {code} ({len(keep)} bound tensors)")
    return launch


def fir_am_i8_carry(taps: torch.Tensor, iq: torch.Tensor, decimation: int, num_outputs: int,
                    out: torch.Tensor, carry: torch.Tensor) -> torch.Tensor:
    """Streaming int8 IQ -> FIR -> AM (gsdrInt8FirFCAmDemodCarry): writes `num_outputs` AM
    samples to `out` and, in the same launch, copies the history the next call needs (the last
    T - D input samples) to `carry`, which may be a view of the start of `iq` (in-place history)."""
    _require(taps, torch.float32, "taps")
    _require(iq, torch.int8, "iq")
    _require(out, torch.float32, "out")
    _require(carry, torch.int8, "carry")
    d = max(1, int(decimation))
    T = taps.numel()
    if num_outputs > 0 and (num_outputs - 1) * d + T > iq.numel() // 2:
        raise ValueError("input too short for the requested outputs")
    if out.numel() < num_outputs or carry.numel() < 2 * max(0, T - d):
        raise ValueError("out or carry too small")
    check(lib().gsdrInt8FirFCAmDemodCarry(d, taps.data_ptr(), T, iq.data_ptr(), out.data_ptr(), num_outputs,
                                          carry.data_ptr(), _dev(iq), _stream(iq)), "gsdrInt8FirFCAmDemodCarry")
    return out


def am_chain_fused(taps: torch.Tensor, iq: torch.Tensor, decimation: int, rf_count: int,
                   am_window: torch.Tensor, am_history: int, audio_taps: torch.Tensor, audio_decimation: int,
                   audio_count: int, audio_out: torch.Tensor, store_am: bool = True) -> torch.Tensor:
    """int8 IQ -> FIR -> AM -> audio FIR in one launch (gsdrInt8FirFCAmDemodFirFF): `rf_count` AM
    samples land in am_window[am_history:] (unless store_am is False: then that part is scratch) and
    `audio_count` audio samples of the FF FIR over am_window = [history | new AM] in `audio_out`."""
    _require(taps, torch.float32, "taps")
    _require(iq, torch.int8, "iq")
    _require(am_window, torch.float32, "am_window")
    _require(audio_taps, torch.float32, "audio_taps")
    _require(audio_out, torch.float32, "audio_out")
    d, da = max(1, int(decimation)), max(1, int(audio_decimation))
    T, Ta = taps.numel(), audio_taps.numel()
    if rf_count > 0 and (rf_count - 1) * d + T > iq.numel() // 2:
        raise ValueError("input too short for the requested RF outputs")
    if am_window.numel() < am_history + rf_count or audio_out.numel() < audio_count:
        raise ValueError("am_window or audio_out too small")
    if audio_count > 0 and (audio_count - 1) * da + Ta > am_history + rf_count:
        raise ValueError("audio outputs need more AM samples than history + rf_count")
    check(lib().gsdrInt8FirFCAmDemodFirFF(d, taps.data_ptr(), T, iq.data_ptr(), rf_count, am_window.data_ptr(),
                                          am_history, 1 if store_am else 0, da, audio_taps.data_ptr(), Ta,
                                          audio_out.data_ptr(), audio_count, _dev(iq), _stream(iq)),
          "gsdrInt8FirFCAmDemodFirFF")
    return audio_out


def poison_lds(device: int = 0, pattern: int = 0x7FC00000, stream=None) -> None:
    """gsdrAmdPoisonLds on `stream` (a torch stream; default: the current stream) - tests: stale-LDS
    reads become visible."""
    s = torch.cuda.current_stream(device) if stream is None else stream
    check(lib().gsdrAmdPoisonLds(pattern, device, ctypes.c_void_p(s.cuda_stream)), "gsdrAmdPoisonLds")


def hbm_probe(src: torch.Tensor, dst: torch.Tensor, mode: int) -> None:
    """gsdrAmdHbmProbe: mode 0 streams src (read bandwidth), mode 1 copies src -> dst."""
    if not (src.is_cuda and dst.is_cuda and src.is_contiguous() and dst.is_contiguous()):
        raise ValueError("contiguous device tensors")
    n = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() < n:
        raise ValueError("dst too small")
    check(lib().gsdrAmdHbmProbe(src.data_ptr(), dst.data_ptr(), n, int(mode), _dev(src), _stream(src)),
          "gsdrAmdHbmProbe")


def copy_kernel(dst: torch.Tensor, src: torch.Tensor) -> None:
    """gsdrAmdCopyKernel on the current stream: src's bytes to dst by a copy kernel (dword-aligned
    addresses and size; device or host-mapped memory)."""
    n = src.numel() * src.element_size()
    if dst.numel() * dst.element_size() < n:
        raise ValueError("dst too small")
    L = lib()
    L.gsdrAmdCopyKernel.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
    dev = dst if dst.is_cuda else src
    check(L.gsdrAmdCopyKernel(dst.data_ptr(), src.data_ptr(), n, _stream(dev)), "gsdrAmdCopyKernel")


def quad_am_demod(z: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    _require(z, torch.complex64, "z")
    if out is None:
        out = torch.empty(z.numel(), dtype=torch.float32, device=z.device)
    check(lib().gsdrQuadAmDemod(z.data_ptr(), out.data_ptr(), z.numel(), _dev(z), _stream(z)), "gsdrQuadAmDemod")
    return out


def multiply_cc(a: torch.Tensor, b: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    """gsdrMultiplyCC: element-wise non-conjugate complex product (MultiplyCcc)."""
    _require(a, torch.complex64, "a")
    _require(b, torch.complex64, "b")
    n = min(a.numel(), b.numel())
    if out is None:
        out = torch.empty(n, dtype=torch.complex64, device=a.device)
    check(lib().gsdrMultiplyCC(a.data_ptr(), b.data_ptr(), out.data_ptr(), n, _dev(a), _stream(a)), "gsdrMultiplyCC")
    return out


def quad_fm_demod(z: torch.Tensor, gain: float, out: torch.Tensor | None = None) -> torch.Tensor:
    """gsdrQuadFmDemod: len(z) - 1 outputs gain * arg(z[i+1] conj(z[i]))."""
    _require(z, torch.complex64, "z")
    n = max(z.numel() - 1, 0)
    if out is None:
        out = torch.empty(n, dtype=torch.float32, device=z.device)
    check(lib().gsdrQuadFmDemod(z.data_ptr(), out.data_ptr(), float(gain), n, _dev(z), _stream(z)),
          "gsdrQuadFmDemod")
    return out


def int8_to_norm_float(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    _require(x, torch.int8, "x")
    if out is None:
        out = torch.empty(x.numel(), dtype=torch.float32, device=x.device)
    check(lib().gsdrInt8ToNormFloat(x.data_ptr(), out.data_ptr(), x.numel(), _dev(x), _stream(x)),
          "gsdrInt8ToNormFloat")
    return out


def float_to_int8(x: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
    _require(x, torch.float32, "x")
    if out is None:
        out = torch.empty(x.numel(), dtype=torch.int8, device=x.device)
    check(lib().gsdrFloatToInt8(x.data_ptr(), out.data_ptr(), x.numel(), _dev(x), _stream(x)), "gsdrFloatToInt8")
    return out


def cosine(phi_begin: float, phi_end: float, n: int, complex_out: bool, device="cuda") -> torch.Tensor:
    dt = torch.complex64 if complex_out else torch.float32
    out = torch.empty(n, dtype=dt, device=device)
    fn = lib().gsdrCosineC if complex_out else lib().gsdrCosineF
    check(fn(phi_begin, phi_end, out.data_ptr(), n, _dev(out), _stream(out)), fn.__name__)
    return out


def synth_iq_int8(seed: int, fs: float, am_hz: float, carrier_hz: float, first: int, n: int,
                  out: torch.Tensor | None = None, device="cuda") -> torch.Tensor:
    if out is None:
        out = torch.empty(2 * n, dtype=torch.int8, device=device)
    check(lib().gsdrSynthIqInt8(seed, fs, am_hz, carrier_hz, first, out.data_ptr(), n, _dev(out), _stream(out)),
          "gsdrSynthIqInt8")
    return out


def synth_wideband_cf32(seed: int, f1: float, f2: float, first: int, n: int,
                        out: torch.Tensor | None = None, device="cuda") -> torch.Tensor:
    if out is None:
        out = torch.empty(n, dtype=torch.complex64, device=device)
    check(lib().gsdrSynthWidebandCf32(seed, f1, f2, first, out.data_ptr(), n, _dev(out), _stream(out)),
          "gsdrSynthWidebandCf32")
    return out


POLICY_NO_MFMA = 1  # include/gsdr/gsdr_amd.h GSDR_POLICY_NO_MFMA
POLICY_CF_BF16 = 2  # GSDR_POLICY_CF_BF16
POLICY_NO_WS = 4  # GSDR_POLICY_NO_WS: barrier-synchronous decimating MFMA kernels
POLICY_NO_FFT = 8  # GSDR_POLICY_NO_FFT: long real-tap FIRs on the direct forms, not the FFT kernel
POLICY_PREFER_FFT = 16  # GSDR_POLICY_PREFER_FFT: the FFT kernel wherever eligible (int8 IQ, small cf32 launches)
POLICY_I8_WS8 = 64  # GSDR_POLICY_I8_WS8: int8 decimating FIRs on the r04 8-way wave-specialised kernel


def kernel_policy() -> int:
    """The process-wide kernel-selection policy flags (gsdrAmdGetKernelPolicy)."""
    L = lib()
    L.gsdrAmdGetKernelPolicy.restype = ctypes.c_uint32
    return int(L.gsdrAmdGetKernelPolicy())


def set_kernel_policy(flags: int) -> int:
    """Set the process-wide kernel-selection policy; returns the previous flags."""
    L = lib()
    L.gsdrAmdGetKernelPolicy.restype = ctypes.c_uint32
    L.gsdrAmdSetKernelPolicy.argtypes = [ctypes.c_uint32]
    prev = L.gsdrAmdGetKernelPolicy()
    L.gsdrAmdSetKernelPolicy(flags)
    return prev


def set_fft_guard(ratio: float) -> float:
    """FFT FIR accuracy guard (gsdrAmdSetFftGuard): blocks whose loudest row exceeds `ratio` times
    the quietest run in the direct fp32 form; 0 forces the direct form. Returns the previous value."""
    L = lib()
    L.gsdrAmdGetFftGuard.restype = ctypes.c_float
    L.gsdrAmdSetFftGuard.argtypes = [ctypes.c_float]
    prev = L.gsdrAmdGetFftGuard()
    L.gsdrAmdSetFftGuard(float(ratio))
    return prev


def fft_direct_blocks(device: int = 0, reset: bool = True) -> int:
    """Blocks the FFT FIR sent to its direct-form fallback since the last reset (syncs the device)."""
    L = lib()
    L.gsdrAmdFftDirectBlocks.argtypes = [ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    L.gsdrAmdFftDirectBlocks.restype = ctypes.c_int
    v = ctypes.c_uint64()
    check(L.gsdrAmdFftDirectBlocks(device, ctypes.byref(v), 1 if reset else 0), "gsdrAmdFftDirectBlocks")
    return int(v.value)


def fir_kernel_class(x: torch.Tensor, taps: torch.Tensor, decimation: int, int8_iq: bool = False) -> str:
    """The kernel family the FC FIR dispatch picks for this input / shape (gsdrAmdFirKernelClass)."""
    L = lib()
    L.gsdrAmdFirKernelClass.argtypes = [ctypes.c_int, ctypes.c_size_t, ctypes.c_size_t, ctypes.c_void_p]
    L.gsdrAmdFirKernelClass.restype = ctypes.c_char_p
    return L.gsdrAmdFirKernelClass(1 if int8_iq else 0, taps.numel(), max(1, int(decimation)),
                                   x.data_ptr()).decode()


def set_ws_spin_limit(microseconds: int) -> int:
    """Hand-off wait budget of the wave-specialised MFMA kernels in microseconds of wall clock
    (gsdrAmdSetWsSpinLimit; 0: give up at the first pending poll); returns the previous value."""
    L = lib()
    L.gsdrAmdGetWsSpinLimit.restype = ctypes.c_int32
    L.gsdrAmdSetWsSpinLimit.argtypes = [ctypes.c_int32]
    prev = L.gsdrAmdGetWsSpinLimit()
    L.gsdrAmdSetWsSpinLimit(int(microseconds))
    return prev


def ws_aborts(device: int = 0, reset: bool = True) -> int:
    """Wave-specialised launches whose hand-off waits gave up since the last reset (gsdrAmdWsAborts;
    synchronises the device). Such launches' outputs are undefined."""
    L = lib()
    L.gsdrAmdWsAborts.argtypes = [ctypes.c_int32, ctypes.POINTER(ctypes.c_uint64), ctypes.c_int]
    L.gsdrAmdWsAborts.restype = ctypes.c_int
    v = ctypes.c_uint64()
    check(L.gsdrAmdWsAborts(device, ctypes.byref(v), 1 if reset else 0), "gsdrAmdWsAborts")
    return int(v.value)


def fm_front(taps: torch.Tensor, x: torch.Tensor, decimation: int, num_outputs: int, phase0: float,
             radians_per_sample: float, gain: float, int8_iq: bool = False,
             out: torch.Tensor | None = None) -> torch.Tensor:
    """Fused FM front (gsdrMixFirFCFmDemod / gsdrInt8MixFirFCFmDemod): mix, low-pass + decimate,
    discriminate in one kernel. Needs num_outputs * D + T input samples."""
    _require(taps, torch.float32, "taps")
    _require(x, torch.int8 if int8_iq else torch.complex64, "x")
    n_in = x.numel() // 2 if int8_iq else x.numel()
    d = max(1, int(decimation))
    if num_outputs > 0 and num_outputs * d + taps.numel() > n_in:
        raise ValueError("input too short for the requested outputs")
    if out is None:
        out = torch.empty(num_outputs, dtype=torch.float32, device=x.device)
    fn = lib().gsdrInt8MixFirFCFmDemod if int8_iq else lib().gsdrMixFirFCFmDemod
    fn.argtypes = [ctypes.c_size_t, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_double,
                   ctypes.c_double, ctypes.c_float, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_void_p]
    check(fn(d, taps.data_ptr(), taps.numel(), x.data_ptr(), float(phase0), float(radians_per_sample), float(gain),
             out.data_ptr(), num_outputs, _dev(x), _stream(x)), fn.__name__)
    return out


def fm_demod(rf_sample_rate: int, tuned: float, channel: float, deviation: float, decimation: int,
             first_sample_offset: int, taps: torch.Tensor, x: torch.Tensor, num_outputs: int) -> torch.Tensor:
    """The reference's gsdrFmDemod (fm_simpletest.cpp:400-413 call site)."""
    out = torch.empty(num_outputs, dtype=torch.float32, device=x.device)
    fn = lib().gsdrFmDemod
    fn.argtypes = [ctypes.c_size_t, ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_size_t, ctypes.c_size_t,
                   ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                   ctypes.c_int32, ctypes.c_void_p]
    check(fn(int(rf_sample_rate), float(tuned), float(channel), float(deviation), int(decimation),
             int(first_sample_offset), taps.data_ptr(), taps.numel(), x.data_ptr(), out.data_ptr(), num_outputs,
             _dev(x), _stream(x)), "gsdrFmDemod")
    return out
