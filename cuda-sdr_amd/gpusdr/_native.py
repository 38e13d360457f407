"""Loader for libgpusdrpipeline.so (the HIP kernels + C++ runtime + flat C API).

The product path has no CPU fallback: if the library is missing or fails to load this raises.
torch is imported first on purpose: torch ships its own libamdhip64.so (soname
libamdhip64.so.7); loading it before our library makes the dynamic linker resolve our
NEEDED libamdhip64.so.7 to that same runtime, so device pointers and streams are shared.
"""
from __future__ import annotations

import ctypes
import os

import torch  # noqa: F401  (must precede the CDLL, see module docstring)

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.normpath(os.path.join(PKG_DIR, "..", "lib", "libgpusdrpipeline.so"))
# A/B builds of the library (tools/exp) may be named here; the in-tree build is the default.
LIB_PATH = os.environ.get("GSDR_LIB") or LIB_PATH

_lib = None


class HipError(RuntimeError):
    pass


def lib() -> ctypes.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(
                f"{LIB_PATH} is missing: build it with `make -C cuda-sdr_amd` "
                "(or __graft_entry__.build()); there is no CPU fallback")
        L = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
        _declare(L)
        _lib = L
    return _lib


def _declare(L):
    sz, vp, f32, f64, i32, u64 = (ctypes.c_size_t, ctypes.c_void_p, ctypes.c_float, ctypes.c_double,
                                  ctypes.c_int32, ctypes.c_uint64)
    err = ctypes.c_int
    fir_sig = [sz, vp, sz, vp, vp, sz, i32, vp]
    for name in ("gsdrFirFF", "gsdrFirFC", "gsdrFirCC", "gsdrFirCF", "gsdrFirFCAmDemod", "gsdrFirCCAmDemod",
                 "gsdrInt8FirFC", "gsdrInt8FirFCAmDemod"):
        fn = getattr(L, name)
        fn.argtypes = fir_sig
        fn.restype = err
    L.gsdrInt8FirFCAmDemodCarry.argtypes = [sz, vp, sz, vp, vp, sz, vp, i32, vp]
    L.gsdrInt8FirFCAmDemodCarry.restype = err
    L.gsdrInt8FirFCAmDemodFirFF.argtypes = [sz, vp, sz, vp, sz, vp, sz, i32, sz, vp, sz, vp, sz, i32, vp]
    L.gsdrInt8FirFCAmDemodFirFF.restype = err
    for name in ("gsdrQuadAmDemod", "gsdrInt8ToNormFloat", "gsdrFloatToInt8"):
        fn = getattr(L, name)
        fn.argtypes = [vp, vp, sz, i32, vp]
        fn.restype = err
    for name in ("gsdrCosineF", "gsdrCosineC"):
        fn = getattr(L, name)
        fn.argtypes = [f32, f32, vp, sz, i32, vp]
        fn.restype = err
    for name in ("gsdrMixFirFC", "gsdrMixFirFCAmDemod", "gsdrInt8MixFirFC", "gsdrInt8MixFirFCAmDemod"):
        fn = getattr(L, name)
        fn.argtypes = [sz, vp, sz, vp, f64, f64, vp, sz, i32, vp]
        fn.restype = err
    L.gsdrMultiplyCC.argtypes = [vp, vp, vp, sz, i32, vp]
    L.gsdrMultiplyCC.restype = err
    L.gsdrQuadFmDemod.argtypes = [vp, vp, f32, sz, i32, vp]
    L.gsdrQuadFmDemod.restype = err
    L.gsdrSynthIqInt8.argtypes = [u64, f64, f64, f64, u64, vp, sz, i32, vp]
    L.gsdrSynthIqInt8.restype = err
    L.gsdrSynthWidebandCf32.argtypes = [u64, f64, f64, u64, vp, sz, i32, vp]
    L.gsdrSynthWidebandCf32.restype = err
    L.gsdrAmdHbmProbe.argtypes = [vp, vp, sz, i32, i32, vp]
    L.gsdrAmdHbmProbe.restype = err
    L.gsdrAmdPoisonLds.argtypes = [ctypes.c_uint32, i32, vp]
    L.gsdrAmdPoisonLds.restype = err
    L.gsdrAmdBuildId.argtypes = []
    L.gsdrAmdBuildId.restype = ctypes.c_char_p


def check(code: int, what: str) -> None:
    if code != 0:
        raise HipError(f"{what} failed with hipError_t {code}")
