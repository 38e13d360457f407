"""Python handles over the gpusdrpipeline filter graph (flat C API, include/gsdr/gpusdr_flat.h).

Mirrors the reference's node interface (src/filters/Fir.cpp etc.): nodes are created through
the factories, fed through Sink.requestBuffer/commitBuffer (``push``) and drained through
Source.readOutput into device buffers (``read``). Every call lands in libgpusdrpipeline.so.
"""
from __future__ import annotations

import ctypes

import numpy as np

from ._native import lib

SAMPLE_FLOAT_COMPLEX, SAMPLE_FLOAT, SAMPLE_INT8_COMPLEX = 0, 1, 2
STATUS_NAMES = ["Success", "UnknownError", "OutOfMemory", "RuntimeError", "InvalidArgument", "InvalidState",
                "OutOfRange", "TimedOut", "NotFound", "ParseError"]


class GraphError(RuntimeError):
    def __init__(self, status: int, what: str):
        name = STATUS_NAMES[status] if status < len(STATUS_NAMES) else str(status)
        super().__init__(f"{what}: Status_{name}")
        self.status = status


_declared = False


def _L():
    global _declared
    L = lib()
    if not _declared:
        h, sz, u32, vp = ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint32, ctypes.c_void_p
        ph = ctypes.POINTER(ctypes.c_void_p)
        psz = ctypes.POINTER(ctypes.c_size_t)
        sigs = {
            "gspRelease": ([h], None),
            "gspQueueCreate": ([ctypes.c_int32, ph], u32),
            "gspQueueStream": ([h], vp),
            "gspQueueSync": ([h], u32),
            "gspFirCreate": ([u32, u32, sz, vp, sz, h, ph], u32),
            "gspQuadAmDemodCreate": ([h, ph], u32),
            "gspInt8ToFloatCreate": ([h, ph], u32),
            "gspCosineSourceCreate": ([u32, ctypes.c_float, ctypes.c_float, h, ph], u32),
            "gspNamedQueueCreate": ([ctypes.c_char_p, ctypes.c_char_p], u32),
            "gspNamedQueueGet": ([ctypes.c_char_p, ph], u32),
            "gspNodeCreate": ([ctypes.c_char_p, ctypes.c_char_p, ph], u32),
            "gspSinkPushHost": ([h, sz, vp, sz, h], u32),
            "gspSinkPushDevice": ([h, sz, vp, sz, h], u32),
            "gspSinkPreferredInputSize": ([h, sz, psz], u32),
            "gspSourceOutputSize": ([h, sz, psz, psz], u32),
            "gspSourceRead": ([h, ph, sz], u32),
            "gspBufferCreate": ([h, sz, ph], u32),
            "gspHostBufferCreate": ([h, sz, ph], u32),
            "gspHostSinkCreate": ([h, ph], u32),
            "gspDeviceSinkCreate": ([h, sz, ph], u32),
            "gspDriverSetFuseFirAm": ([h, ctypes.c_int32], u32),
            "gspDriverFusedSteps": ([h, psz], u32),
            "gspHostSinkAvailable": ([h, psz], u32),
            "gspHostSinkRead": ([h, vp, sz, psz], u32),
            "gspHostSinkFlush": ([h], u32),
            "gspDesignLowPass": ([ctypes.c_double] * 4 + [vp, sz, psz], u32),
            "gspBufferSlice": ([h, sz, sz, ph], u32),
            "gspBufferRange": ([h, psz, psz, psz], u32),
            "gspBufferSetRange": ([h, sz, sz], u32),
            "gspBufferBase": ([h], vp),
            "gspBufferToHost": ([h, vp, sz, h], u32),
            "gspSteppingDriverCreate": ([ph], u32),
            "gspDriverConnect": ([h, h, sz, h, sz], u32),
            "gspDriverSetupNode": ([h, h, ctypes.c_char_p], u32),
            "gspDriverDoFilter": ([h], u32),
            "gspDriverDoFilterGraphed": ([h, h], u32),
            "gspDriverGraphStats": ([h, psz, psz, psz], u32),
            "gspDriverGraphDirectReplays": ([h, psz], u32),
            "gspDriverNodeName": ([h, h, ctypes.c_char_p, sz, ctypes.POINTER(ctypes.c_int32)], sz),
        }
        for name, (args, res) in sigs.items():
            fn = getattr(L, name)
            fn.argtypes = args
            fn.restype = res
        _declared = True
    return L


def _check(status, what):
    if status != 0:
        raise GraphError(status, what)


class _Handle:
    def __init__(self, ptr):
        self._h = ctypes.c_void_p(ptr)

    @property
    def handle(self):
        return self._h

    def release(self):
        if self._h:
            _L().gspRelease(self._h)
            self._h = ctypes.c_void_p(None)

    def __del__(self):
        try:
            self.release()
        except Exception:
            pass


def _create(fn, *args, what=""):
    out = ctypes.c_void_p()
    _check(fn(*args, ctypes.byref(out)), what)
    return out.value


class Queue(_Handle):
    """ICudaCommandQueue: one HIP device + one non-blocking stream."""

    def __init__(self, device: int = 0, _ptr=None):
        super().__init__(_ptr if _ptr is not None else _create(_L().gspQueueCreate, device, what="gspQueueCreate"))

    @classmethod
    def named(cls, name: str, device: int = 0) -> "Queue":
        """Create (or reuse) the named queue JSON nodes refer to ({"commandQueue": name})."""
        st = _L().gspNamedQueueCreate(name.encode(), f'{{"queueType": "hip", "cudaDevice": {device}}}'.encode())
        if st not in (0, 5):  # Status_InvalidState: the name exists already
            _check(st, "gspNamedQueueCreate")
        return cls(_ptr=_create(_L().gspNamedQueueGet, name.encode(), what="gspNamedQueueGet"))

    @property
    def stream(self) -> int:
        return _L().gspQueueStream(self._h)

    def sync(self):
        _check(_L().gspQueueSync(self._h), "gspQueueSync")


class Buffer(_Handle):
    """IBuffer over device memory (or a slice of one)."""

    def __init__(self, ptr, queue: Queue, parent=None):
        super().__init__(ptr)
        self.queue = queue
        self._parent = parent

    @classmethod
    def create(cls, queue: Queue, nbytes: int) -> "Buffer":
        return cls(_create(_L().gspBufferCreate, queue.handle, nbytes, what="gspBufferCreate"), queue)

    @classmethod
    def create_host(cls, queue: Queue, nbytes: int) -> "Buffer":
        """Pinned host memory (the output side of a device -> host staging filter)."""
        return cls(_create(_L().gspHostBufferCreate, queue.handle, nbytes, what="gspHostBufferCreate"), queue)

    def slice(self, start: int, end: int) -> "Buffer":
        return Buffer(_create(_L().gspBufferSlice, self._h, start, end, what="gspBufferSlice"), self.queue, self)

    def range(self):
        o, e, c = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        _check(_L().gspBufferRange(self._h, ctypes.byref(o), ctypes.byref(e), ctypes.byref(c)), "gspBufferRange")
        return o.value, e.value, c.value

    def used(self) -> int:
        o, e, _ = self.range()
        return e - o

    def set_range(self, offset: int, end: int):
        _check(_L().gspBufferSetRange(self._h, offset, end), "gspBufferSetRange")

    def clear(self):
        self.set_range(0, 0)

    def to_host(self, dtype) -> np.ndarray:
        n = self.used()
        out = np.empty(n, dtype=np.uint8)
        _check(_L().gspBufferToHost(self._h, out.ctypes.data, n, self.queue.handle), "gspBufferToHost")
        return out.view(dtype)


def design_lowpass(sample_rate: float, cutoff: float, transition: float, db_attenuation: float) -> np.ndarray:
    """The RF -> PCM component's low-pass designer (gspDesignLowPass; Kaiser window at the
    reference's fred harris length)."""
    n = ctypes.c_size_t()
    _check(_L().gspDesignLowPass(sample_rate, cutoff, transition, db_attenuation, None, 0, ctypes.byref(n)),
           "gspDesignLowPass")
    taps = np.empty(n.value, dtype=np.float32)
    _check(_L().gspDesignLowPass(sample_rate, cutoff, transition, db_attenuation, taps.ctypes.data, len(taps),
                                 ctypes.byref(n)), "gspDesignLowPass")
    return taps


class Node(_Handle):
    """A Filter / Source / Sink of the reference object model."""

    def __init__(self, ptr, queue: Queue | None):
        super().__init__(ptr)
        self.queue = queue

    def graph_stats(self):
        """A JSON Component's inner stepping: plain, capturing and replayed steps (hipGraph)."""
        e, c, r, d = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_size_t()
        _check(_L().gspDriverGraphStats(self._h, ctypes.byref(e), ctypes.byref(c), ctypes.byref(r)), "graphStats")
        _check(_L().gspDriverGraphDirectReplays(self._h, ctypes.byref(d)), "graphDirectReplays")
        return {"eager": e.value, "captured": c.value, "replayed": r.value, "direct": d.value}

    # -- constructors mirroring the reference factories --
    @classmethod
    def fir(cls, queue: Queue, taps: np.ndarray, decimation: int = 1, element_type: int = SAMPLE_FLOAT_COMPLEX):
        taps_c = np.iscomplexobj(taps)
        t = np.ascontiguousarray(taps, dtype=np.complex64 if taps_c else np.float32)
        tap_type = SAMPLE_FLOAT_COMPLEX if taps_c else SAMPLE_FLOAT
        return cls(_create(_L().gspFirCreate, tap_type, element_type, decimation, t.ctypes.data, len(t), queue.handle,
                           what="gspFirCreate"), queue)

    @classmethod
    def quad_am_demod(cls, queue: Queue):
        return cls(_create(_L().gspQuadAmDemodCreate, queue.handle, what="gspQuadAmDemodCreate"), queue)

    @classmethod
    def host_sink(cls, queue: Queue):
        """The host egress sink (gspHostSinkCreate): one step in flight, the rest in a host FIFO."""
        return cls(_create(_L().gspHostSinkCreate, queue.handle, what="gspHostSinkCreate"), queue)

    @classmethod
    def device_sink(cls, queue: Queue, preferred_bytes: int = 0):
        """A device sink that retires every committed byte (gspDeviceSinkCreate)."""
        return cls(_create(_L().gspDeviceSinkCreate, queue.handle, preferred_bytes, what="gspDeviceSinkCreate"),
                   queue)

    def host_available(self):
        n = ctypes.c_size_t()
        _check(_L().gspHostSinkAvailable(self._h, ctypes.byref(n)), "hostSinkAvailable")
        return n.value

    def host_read(self, dtype, max_bytes=None):
        """Drain the host sink's FIFO as an array of `dtype`."""
        cap = self.host_available() if max_bytes is None else max_bytes
        out = np.empty(cap, dtype=np.uint8)
        n = ctypes.c_size_t()
        _check(_L().gspHostSinkRead(self._h, out.ctypes.data_as(ctypes.c_void_p), cap, ctypes.byref(n)),
               "hostSinkRead")
        return out[:n.value].view(dtype)

    def host_flush(self):
        _check(_L().gspHostSinkFlush(self._h), "hostSinkFlush")

    @classmethod
    def int8_to_float(cls, queue: Queue):
        return cls(_create(_L().gspInt8ToFloatCreate, queue.handle, what="gspInt8ToFloatCreate"), queue)

    @classmethod
    def cosine(cls, queue: Queue, sample_type: int, sample_rate: float, frequency: float):
        return cls(_create(_L().gspCosineSourceCreate, sample_type, sample_rate, frequency, queue.handle,
                           what="gspCosineSourceCreate"), queue)

    @classmethod
    def from_json(cls, name: str, params: str, queue: Queue | None = None):
        return cls(_create(_L().gspNodeCreate, name.encode(), params.encode(), what=f"createNode({name})"), queue)

    # -- Sink --
    def push(self, data: np.ndarray, port: int = 0):
        a = np.ascontiguousarray(data)
        _check(_L().gspSinkPushHost(self._h, port, a.ctypes.data, a.nbytes, self.queue.handle), "push")

    def push_device(self, ptr: int, nbytes: int, port: int = 0):
        _check(_L().gspSinkPushDevice(self._h, port, ptr, nbytes, self.queue.handle), "push_device")

    def preferred_input_size(self, port: int = 0) -> int:
        n = ctypes.c_size_t()
        _check(_L().gspSinkPreferredInputSize(self._h, port, ctypes.byref(n)), "preferredInputBufferSize")
        return n.value

    # -- Source --
    def output_size(self, port: int = 0):
        n, a = ctypes.c_size_t(), ctypes.c_size_t()
        _check(_L().gspSourceOutputSize(self._h, port, ctypes.byref(n), ctypes.byref(a)), "getOutputDataSize")
        return n.value, a.value

    def read(self, buffers):
        arr = (ctypes.c_void_p * len(buffers))(*[b.handle.value for b in buffers])
        _check(_L().gspSourceRead(self._h, arr, len(buffers)), "readOutput")


class SteppingDriver(_Handle):
    """ISteppingDriver (reference src/driver/SteppingDriver.cpp): connect nodes, then each
    ``do_filter()`` pulls one chunk through every graph tail's upstream chain. Holds references
    to the nodes it connects."""

    def __init__(self):
        super().__init__(_create(_L().gspSteppingDriverCreate, what="createSteppingDriver"))
        self._nodes = []

    def connect(self, source: Node, source_port: int, sink: Node, sink_port: int = 0):
        _check(_L().gspDriverConnect(self._h, source.handle, source_port, sink.handle, sink_port), "connect")
        self._nodes += [source, sink]

    def setup_node(self, node: Node, name: str):
        _check(_L().gspDriverSetupNode(self._h, node.handle, name.encode()), "setupNode")

    def node_name(self, node: Node):
        found = ctypes.c_int32()
        buf = ctypes.create_string_buffer(256)
        n = _L().gspDriverNodeName(self._h, node.handle, buf, len(buf), ctypes.byref(found))
        return buf.raw[:min(n, 255)].decode() if found.value else None

    def do_filter(self):
        _check(_L().gspDriverDoFilter(self._h), "doFilter")

    def do_filter_graphed(self, queue: Queue):
        """One step with its device work replayed from a hipGraph captured per repeating chain
        state (gspDriverDoFilterGraphed); a plain step when the chain cannot be replayed."""
        _check(_L().gspDriverDoFilterGraphed(self._h, queue.handle), "doFilterGraphed")

    def graph_stats(self):
        e, c, r, f, d = (ctypes.c_size_t() for _ in range(5))
        _check(_L().gspDriverGraphStats(self._h, ctypes.byref(e), ctypes.byref(c), ctypes.byref(r)), "graphStats")
        _check(_L().gspDriverFusedSteps(self._h, ctypes.byref(f)), "fusedSteps")
        _check(_L().gspDriverGraphDirectReplays(self._h, ctypes.byref(d)), "graphDirectReplays")
        return {"eager": e.value, "captured": c.value, "replayed": r.value, "fused": f.value, "direct": d.value}

    def set_fuse_fir_am(self, on: bool):
        """Fir -> QuadAmDemod as one fused launch (default on; off = the reference's two launches)."""
        _check(_L().gspDriverSetFuseFirAm(self._h, 1 if on else 0), "setFuseFirAm")
