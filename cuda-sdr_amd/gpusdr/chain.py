"""AM receive chain executor (gsdrAmChain*, include/gsdr/gsdr_amd.h): int8 IQ -> cf32 -> FC FIR ->
AM -> FF FIR, one hipGraph launch per fixed-size chunk. Thin ctypes plumbing; no CPU path."""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ._native import check, lib


class _Config(ctypes.Structure):
    _fields_ = [("rfTaps", ctypes.c_void_p), ("rfTapCount", ctypes.c_size_t), ("rfDecimation", ctypes.c_size_t),
                ("audioTaps", ctypes.c_void_p), ("audioTapCount", ctypes.c_size_t),
                ("audioDecimation", ctypes.c_size_t), ("chunkSamples", ctypes.c_size_t),
                ("hostSlots", ctypes.c_size_t)]


_declared = False


def _L():
    global _declared
    L = lib()
    if not _declared:
        vp, sz, err = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int
        psz = ctypes.POINTER(ctypes.c_size_t)
        for name, args, res in (
                ("gsdrAmChainCreate", [ctypes.POINTER(_Config), ctypes.c_int32, ctypes.POINTER(vp)], err),
                ("gsdrAmChainDestroy", [vp], None),
                ("gsdrAmChainStream", [vp], vp),
                ("gsdrAmChainNextOutputCount", [vp], sz),
                ("gsdrAmChainStep", [vp, vp, vp, psz], err),
                ("gsdrAmChainHostInputSlot", [vp, sz], vp),
                ("gsdrAmChainHostOutputSlot", [vp, sz], vp),
                ("gsdrAmChainStepHost", [vp, sz, psz], err),
                ("gsdrAmChainWaitSlot", [vp, sz], err),
                ("gsdrAmChainReset", [vp], err),
                ("gsdrAmChainResidentOutputCount", [vp, sz], sz),
                ("gsdrAmChainStepResident", [vp, vp, sz, vp, psz], err),
                ("gsdrAmChainChunksOutputCount", [vp, sz], sz),
                ("gsdrAmChainStepChunks", [vp, vp, sz, vp, psz], err),
                ("gsdrAmChainGraphCaptures", [vp], sz)):
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _declared = True
    return L


class AmChain:
    """One chain on one device. ``step(iq)`` takes a device int8 tensor of 2*chunk values and
    returns the audio samples of that step (device float32 tensor)."""

    def __init__(self, rf_taps, rf_decimation, audio_taps, audio_decimation, chunk_samples, device=0,
                 host_slots=0):
        self.rf_taps = np.ascontiguousarray(rf_taps, dtype=np.float32)
        self.audio_taps = np.ascontiguousarray(audio_taps, dtype=np.float32)
        self.chunk = int(chunk_samples)
        self.device = int(device)
        self.slots = int(host_slots)
        cfg = _Config(self.rf_taps.ctypes.data, len(self.rf_taps), int(rf_decimation), self.audio_taps.ctypes.data,
                      len(self.audio_taps), int(audio_decimation), self.chunk, self.slots)
        h = ctypes.c_void_p()
        check(_L().gsdrAmChainCreate(ctypes.byref(cfg), self.device, ctypes.byref(h)), "gsdrAmChainCreate")
        self._h = h
        self.torch_stream = torch.cuda.ExternalStream(_L().gsdrAmChainStream(h), device=f"cuda:{self.device}")

    def close(self):
        if self._h:
            _L().gsdrAmChainDestroy(self._h)
            self._h = ctypes.c_void_p(None)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def next_output_count(self) -> int:
        return _L().gsdrAmChainNextOutputCount(self._h)

    def step(self, iq: torch.Tensor, out: torch.Tensor | None = None) -> torch.Tensor:
        if iq.dtype != torch.int8 or not iq.is_cuda or not iq.is_contiguous() or iq.numel() != 2 * self.chunk:
            raise ValueError("iq must be a contiguous device int8 tensor of 2*chunk values")
        n = self.next_output_count()
        if out is None:
            out = torch.empty(n, dtype=torch.float32, device=iq.device)
        elif out.numel() < n:
            raise ValueError("out too small")
        # the chain's stream must see iq's producer; order it after torch's current stream
        self.torch_stream.wait_stream(torch.cuda.current_stream(iq.device))
        got = ctypes.c_size_t()
        check(_L().gsdrAmChainStep(self._h, iq.data_ptr(), out.data_ptr(), ctypes.byref(got)), "gsdrAmChainStep")
        torch.cuda.current_stream(iq.device).wait_stream(self.torch_stream)
        return out[: got.value]

    def resident_output_count(self, n_chunks: int) -> int:
        return _L().gsdrAmChainResidentOutputCount(self._h, n_chunks)

    def step_resident(self, iq: torch.Tensor, n_chunks: int, out: torch.Tensor) -> int:
        """n_chunks chunks starting at iq (a view into a contiguous stream buffer: after the first
        step the RF history is read from the samples in front of it). Returns the audio count."""
        if iq.dtype != torch.int8 or not iq.is_cuda or iq.numel() < 2 * self.chunk * n_chunks:
            raise ValueError("iq must be a device int8 view of n_chunks chunks")
        n = self.resident_output_count(n_chunks)
        if out.numel() < n:
            raise ValueError("out too small")
        self.torch_stream.wait_stream(torch.cuda.current_stream(iq.device))
        got = ctypes.c_size_t()
        check(_L().gsdrAmChainStepResident(self._h, iq.data_ptr(), n_chunks, out.data_ptr(), ctypes.byref(got)),
              "gsdrAmChainStepResident")
        torch.cuda.current_stream(iq.device).wait_stream(self.torch_stream)
        return got.value

    def chunks_output_count(self, n_chunks: int) -> int:
        return _L().gsdrAmChainChunksOutputCount(self._h, n_chunks)

    def step_chunks(self, iq: torch.Tensor, n_chunks: int, out: torch.Tensor) -> int:
        """n_chunks live-stream chunk steps as ONE cached graph launch, output identical to n_chunks
        step() calls; the audio of all of them lands contiguously in out. Chunks 1.. are read in
        place, so iq must stay unmodified until the chain stream has run the launch. Returns the
        audio count."""
        if iq.dtype != torch.int8 or not iq.is_cuda or iq.numel() < 2 * self.chunk * n_chunks:
            raise ValueError("iq must be a device int8 tensor of n_chunks chunks")
        n = self.chunks_output_count(n_chunks)
        if out.numel() < n:
            raise ValueError("out too small")
        self.torch_stream.wait_stream(torch.cuda.current_stream(iq.device))
        got = ctypes.c_size_t()
        check(_L().gsdrAmChainStepChunks(self._h, iq.data_ptr(), n_chunks, out.data_ptr(), ctypes.byref(got)),
              "gsdrAmChainStepChunks")
        torch.cuda.current_stream(iq.device).wait_stream(self.torch_stream)
        return got.value

    # -- pinned ring --
    def host_input(self, slot: int) -> np.ndarray:
        p = _L().gsdrAmChainHostInputSlot(self._h, slot)
        if not p:
            raise IndexError(slot)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_int8)), shape=(2 * self.chunk,))

    def step_host(self, slot: int) -> int:
        got = ctypes.c_size_t()
        check(_L().gsdrAmChainStepHost(self._h, slot, ctypes.byref(got)), "gsdrAmChainStepHost")
        return got.value

    def wait_host(self, slot: int, count: int) -> np.ndarray:
        check(_L().gsdrAmChainWaitSlot(self._h, slot), "gsdrAmChainWaitSlot")
        p = _L().gsdrAmChainHostOutputSlot(self._h, slot)
        return np.ctypeslib.as_array(ctypes.cast(p, ctypes.POINTER(ctypes.c_float)), shape=(count,)).copy()

    def reset(self):
        check(_L().gsdrAmChainReset(self._h), "gsdrAmChainReset")

    def graph_captures(self) -> int:
        """Graphs instantiated so far (3 at creation + every StepChunks / StepResident capture)."""
        return _L().gsdrAmChainGraphCaptures(self._h)
