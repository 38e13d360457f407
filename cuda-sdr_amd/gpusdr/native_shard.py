"""Native time-sharded stream (gsdrShardStream*, include/gsdr/gsdr_amd.h): the per-rank halo-ring
step of gpusdr/shard.py run by the C++ executor, with the exchange supplied by the caller (an RCCL
communicator via gsdrShardExchangeRccl, or a Python callable). Thin ctypes plumbing; no CPU path."""
from __future__ import annotations

import ctypes

import numpy as np
import torch

from ._native import check, lib

EXCHANGE_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t,
                               ctypes.c_int32, ctypes.c_int32, ctypes.c_void_p)
_declared = False
_HIP_D2H, _HIP_H2D, _HIP_D2D = 2, 1, 3


def _L():
    global _declared
    L = lib()
    if not _declared:
        vp, sz, i32, err = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int32, ctypes.c_int
        for name, args, res in (
                ("gsdrShardStreamCreate", [i32, i32, i32, i32, vp, sz, sz, sz, EXCHANGE_FN, vp, i32,
                                           ctypes.POINTER(vp)], err),
                ("gsdrShardStreamDestroy", [vp], None),
                ("gsdrShardStreamSegment", [vp], vp),
                ("gsdrShardStreamHalo", [vp], vp),
                ("gsdrShardStreamOutputCount", [vp], sz),
                ("gsdrShardStreamStep", [vp, vp, vp], err),
                ("gsdrShardRcclGetUniqueId", [vp], err),
                ("gsdrShardRcclCommCreate", [i32, vp, i32, i32, ctypes.POINTER(vp)], err),
                ("gsdrShardRcclCommDestroy", [vp], err),
                ("gsdrShardRcclLastResult", [ctypes.POINTER(ctypes.c_char_p)], i32),
                ("gsdrShardExchangeRccl", [vp, vp, vp, sz, i32, i32, vp], err),
                ("hipStreamSynchronize", [vp], err),
                ("hipMemcpy", [vp, vp, sz, ctypes.c_int], err),
                ("hipMemcpyAsync", [vp, vp, sz, ctypes.c_int, vp], err)):
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _declared = True
    return L


def rccl_last_result():
    """(ncclResult_t, RCCL's text) of this thread's last RCCL call through the library."""
    msg = ctypes.c_char_p()
    code = _L().gsdrShardRcclLastResult(ctypes.byref(msg))
    return code, (msg.value or b"").decode()


def _rccl_check(code, what):
    if code != 0:
        res, msg = rccl_last_result()
        raise RuntimeError(f"{what}: hipError_t {code}, last ncclResult_t {res} ({msg})")


class RcclComm:
    """An RCCL communicator made by the library (gsdrShardRcclCommCreate). Rank 0 calls
    ``RcclComm.unique_id()`` and hands the 128 bytes to every rank; ``RcclComm(n, uid, rank, device)``
    on each. Pass it as ShardStream's ``exchange``: the executor then calls gsdrShardExchangeRccl
    itself (grouped ncclSend / ncclRecv of the halo bytes on its exchange stream; no Python hook)."""

    @staticmethod
    def unique_id() -> bytes:
        buf = ctypes.create_string_buffer(128)
        _rccl_check(_L().gsdrShardRcclGetUniqueId(buf), "gsdrShardRcclGetUniqueId")
        return buf.raw

    def __init__(self, nranks: int, uid: bytes, rank: int, device: int = 0):
        if len(uid) != 128:
            raise ValueError("an ncclUniqueId is 128 bytes")
        self._uid = ctypes.create_string_buffer(uid, 128)
        self._users = 0  # ShardStreams whose exchange hook holds this communicator
        self.handle = ctypes.c_void_p(None)
        h = ctypes.c_void_p()
        _rccl_check(_L().gsdrShardRcclCommCreate(int(nranks), self._uid, int(rank), int(device), ctypes.byref(h)),
                    "gsdrShardRcclCommCreate")
        self.handle = h

    def exchange(self, send_tail, recv_halo, nbytes, next_rank, prev_rank, xstream):
        """gsdrShardExchangeRccl on this communicator (enqueued on `xstream`)."""
        _rccl_check(_L().gsdrShardExchangeRccl(self.handle, send_tail, recv_halo, nbytes, next_rank, prev_rank,
                                               xstream), "gsdrShardExchangeRccl")

    def close(self):
        """Destroy the communicator. Refused while a ShardStream still uses it (the executor
        would keep a dangling ncclComm_t, with RCCL work possibly queued on its exchange stream): close
        those streams first."""
        if self._users > 0:
            raise RuntimeError(f"RcclComm.close: {self._users} ShardStream(s) still use this communicator; "
                               "close them first")
        if self.handle:
            _rccl_check(_L().gsdrShardRcclCommDestroy(self.handle), "gsdrShardRcclCommDestroy")
            self.handle = ctypes.c_void_p(None)

    def __del__(self):
        # a ShardStream keeps a reference to its communicator, so by the time this runs none uses it
        try:
            if self._users == 0:
                self.close()
        except Exception:
            pass


def host_staged_exchange(group=None):
    """An exchange callable for ShardStream over a torch.distributed backend that moves host
    tensors (gloo): it synchronises the exchange stream, stages the tail through host memory, sends
    it to the next rank, receives the halo from the previous rank and copies it in before
    returning (so the data is in place for everything enqueued after the exchange)."""
    import torch.distributed as dist

    def exchange(send_tail, recv_halo, nbytes, next_rank, prev_rank, xstream):
        L = _L()
        check(L.hipStreamSynchronize(xstream), "hipStreamSynchronize")
        send = np.empty(nbytes, dtype=np.uint8)
        recv = np.empty(nbytes, dtype=np.uint8)
        check(L.hipMemcpy(send.ctypes.data, send_tail, nbytes, _HIP_D2H), "hipMemcpy D2H")
        reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, torch.from_numpy(send), next_rank, group),
                                       dist.P2POp(dist.irecv, torch.from_numpy(recv), prev_rank, group)])
        for r in reqs:
            r.wait()
        check(L.hipMemcpy(recv_halo, recv.ctypes.data, nbytes, _HIP_H2D), "hipMemcpy H2D")
    return exchange


class ShardStream:
    """One rank's executor. ``write_segment(x)`` stages the next segment (a device tensor of
    seg_len samples: int8 IQ pairs or complex64), ``step()`` runs the sharded step and returns the
    seg_len / D outputs (float32 AM, or complex64)."""

    def __init__(self, rank, world, taps, decimation, seg_len, int8_iq=False, am=True, exchange=None, device=0):
        self.taps = np.ascontiguousarray(taps, dtype=np.float32)
        self.rank, self.world, self.D, self.L = int(rank), int(world), int(decimation), int(seg_len)
        self.int8_iq, self.am, self.device = bool(int8_iq), bool(am), int(device)
        self.elem = 2 if self.int8_iq else 8
        self.halo_samples = len(self.taps) - 1
        self._py_exchange = exchange

        def trampoline(user, send_tail, recv_halo, nbytes, next_rank, prev_rank, xstream):
            try:
                self._py_exchange(send_tail, recv_halo, nbytes, next_rank, prev_rank, xstream)
                return 0
            except Exception:  # noqa: BLE001 - reported to the executor as a failed exchange
                import traceback
                traceback.print_exc()
                return 999  # hipErrorUnknown

        user = None
        self._comm = None
        self._h = ctypes.c_void_p(None)
        if isinstance(exchange, RcclComm):  # the native hook itself, user = the communicator
            if not exchange.handle:
                raise ValueError("ShardStream: the RcclComm is closed")
            self._cb = ctypes.cast(_L().gsdrShardExchangeRccl, EXCHANGE_FN)
            user = exchange.handle
            self._comm = exchange  # kept alive (and its close() refused) until this stream is closed
        else:
            self._cb = EXCHANGE_FN(trampoline) if exchange is not None else EXCHANGE_FN()
        h = ctypes.c_void_p()
        check(_L().gsdrShardStreamCreate(self.rank, self.world, int(self.int8_iq), int(self.am),
                                         self.taps.ctypes.data, len(self.taps), self.D, self.L, self._cb, user,
                                         self.device, ctypes.byref(h)), "gsdrShardStreamCreate")
        self._h = h
        if self._comm is not None:
            self._comm._users += 1
        self.outputs = _L().gsdrShardStreamOutputCount(h)

    def close(self):
        """Destroy the executor (it waits for its own queued steps and exchanges), then release the
        communicator it used."""
        if self._h:
            _L().gsdrShardStreamDestroy(self._h)
            self._h = ctypes.c_void_p(None)
            if self._comm is not None:
                self._comm._users -= 1
                self._comm = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _copy_in(self, dst, x, n):
        nbytes = n * self.elem
        if not x.is_cuda or not x.is_contiguous() or x.numel() * x.element_size() != nbytes:
            raise ValueError(f"expected a contiguous device tensor of {nbytes} bytes")
        stream = torch.cuda.current_stream(x.device)
        check(_L().hipMemcpyAsync(dst, x.data_ptr(), nbytes, _HIP_D2D, stream.cuda_stream), "hipMemcpyAsync")

    @property
    def halo_ptr(self) -> int:
        """Device address of the halo (tapCount - 1 samples in front of the segment)."""
        return _L().gsdrShardStreamHalo(self._h)

    @property
    def tail_ptr(self) -> int:
        """Device address of the segment's last tapCount - 1 samples (what the exchange sends on)."""
        return _L().gsdrShardStreamSegment(self._h) + (self.L - self.halo_samples) * self.elem

    def write_segment(self, x: torch.Tensor):
        self._copy_in(_L().gsdrShardStreamSegment(self._h), x, self.L)

    def write_halo(self, x: torch.Tensor):
        """Prime the halo (tapCount - 1 samples in front of the segment)."""
        self._copy_in(_L().gsdrShardStreamHalo(self._h), x, self.halo_samples)

    def step(self, out: torch.Tensor | None = None) -> torch.Tensor:
        dev = torch.device("cuda", self.device)
        if out is None:
            out = torch.empty(self.outputs, dtype=torch.float32 if self.am else torch.complex64, device=dev)
        stream = torch.cuda.current_stream(dev)
        check(_L().gsdrShardStreamStep(self._h, out.data_ptr(), stream.cuda_stream), "gsdrShardStreamStep")
        return out
