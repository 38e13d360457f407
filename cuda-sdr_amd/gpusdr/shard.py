"""Time-sharding of one sample stream over the ranks of a torch.distributed group.

SURVEY.md 8(e): the FIR is a sliding window, so a long stream shards by time with a halo of
(T - 1) input samples per boundary and no other communication; QuadAmDemod is element-wise.

Layout (weak scaling, one segment of L samples per rank per step):

    step s, rank g owns stream samples  [(s*G + g)*L, (s*G + g + 1)*L)
    its FIR window is  [halo (T-1 samples) | segment (L samples)]  -> L/D outputs

The halo is the tail of the segment that precedes it in stream order: rank g-1's segment of the
same step, or - for rank 0 - rank G-1's segment of the previous step. One ring exchange per
step (every rank sends its tail to g+1) carries every boundary: ranks g > 0 wait for it before
their head outputs; rank 0 receives the halo for its NEXT step, so its head uses the halo that
arrived one step earlier and never waits. At G = 1 the ring degenerates to the single-stream
history carry (the reference keeps the same T-1 samples in its input window between readOutput
calls, Fir.cpp:274-276). Before the first step the halo is zero: the sharded stream equals the
reference Fir fed (T-1) zeros followed by the stream.

The outputs split into a bulk part that needs only the local segment (launched before the
exchange completes, so the exchange overlaps it) and a head of ceil((T-1)/D) outputs that
reads the halo. Decimation phase is preserved because L % D == 0.
"""
from __future__ import annotations

from dataclasses import dataclass


@dataclass(frozen=True)
class ShardGeometry:
    rank: int
    world: int
    seg_len: int     # L: input samples per rank per step
    taps: int        # T
    decimation: int  # D

    def __post_init__(self):
        if self.seg_len % self.decimation != 0:
            raise ValueError("segment length must be a multiple of the decimation")
        if self.seg_len < self.halo:
            raise ValueError("segment shorter than the halo")

    @property
    def halo(self) -> int:
        return self.taps - 1

    @property
    def outputs(self) -> int:
        return self.seg_len // self.decimation

    @property
    def head_outputs(self) -> int:
        """Outputs whose window reaches into the halo: k*D < T-1."""
        return min(self.outputs, -(-self.halo // self.decimation))

    def segment_start(self, step: int) -> int:
        """Stream index of this rank's first segment sample in `step`."""
        return (step * self.world + self.rank) * self.seg_len

    def first_output(self, step: int) -> int:
        """Global index of this rank's first output in `step` (stream fed T-1 zeros first)."""
        return self.segment_start(step) // self.decimation

    def bulk_input_offset(self) -> int:
        """Offset into the segment of the first input of output head_outputs."""
        return self.head_outputs * self.decimation - self.halo

    @property
    def next_rank(self) -> int:
        return (self.rank + 1) % self.world

    @property
    def prev_rank(self) -> int:
        return (self.rank - 1) % self.world


@dataclass(frozen=True)
class ChainShardGeometry:
    """The cascaded halo of the AM receive chain (C5: int8 IQ -> FC FIR (T, D) -> AM -> FF FIR
    (Ta, Da)), SURVEY.md 8(e): an audio output needs Ta - 1 earlier AM samples, each of which needs
    T - 1 earlier inputs, so a segment needs (Ta - 1) D + T - 1 input samples in front of it
    (3 562 at T = 1023, D = 10, Ta = 255), rounded up here to a multiple of D Da so the decimation
    phases of both FIRs are kept (3 600).

    Each rank runs the chain afresh over [halo | segment] every step: RF outputs k (inputs
    [kD, kD + T) of that window) -> AM -> audio outputs; that yields exactly L / (D Da) audio
    samples, the padded stream's outputs from index segment_start / (D Da) on (the stream fed
    `halo` zeros first, as ShardGeometry feeds T - 1 zeros). The RF outputs whose windows start
    in the segment (k >= halo / D) need no halo: the bulk launch runs while the exchange is in
    flight; the head_rf outputs before them read the halo."""
    rank: int
    world: int
    seg_len: int
    taps: int
    decimation: int
    audio_taps: int
    audio_decimation: int

    def __post_init__(self):
        if self.seg_len % (self.decimation * self.audio_decimation) != 0:
            raise ValueError("segment length must be a multiple of D * Da")
        if self.seg_len < self.halo:
            raise ValueError("segment shorter than the halo")
        if self.outputs_of(self.halo + self.seg_len) != self.outputs:
            raise AssertionError("halo does not yield exactly L / (D Da) audio samples")

    @property
    def halo(self) -> int:
        need = (self.audio_taps - 1) * self.decimation + self.taps - 1
        unit = self.decimation * self.audio_decimation
        return -(-need // unit) * unit

    def rf_outputs_of(self, n_in: int) -> int:
        return max(0, (n_in - (self.taps - 1)) // self.decimation)  # Fir.cpp:178-186

    def outputs_of(self, n_in: int) -> int:
        return max(0, (self.rf_outputs_of(n_in) - (self.audio_taps - 1)) // self.audio_decimation)

    @property
    def rf_outputs(self) -> int:
        return self.rf_outputs_of(self.halo + self.seg_len)

    @property
    def head_rf(self) -> int:
        """RF outputs whose input windows start in the halo."""
        return self.halo // self.decimation

    @property
    def outputs(self) -> int:
        return self.seg_len // (self.decimation * self.audio_decimation)

    def segment_start(self, step: int) -> int:
        return (step * self.world + self.rank) * self.seg_len

    def first_output(self, step: int) -> int:
        """Global index (in the halo-zero-padded stream's audio) of this rank's first output."""
        return self.segment_start(step) // (self.decimation * self.audio_decimation)

    @property
    def next_rank(self) -> int:
        return (self.rank + 1) % self.world

    @property
    def prev_rank(self) -> int:
        return (self.rank - 1) % self.world


def _bytes(t):
    """The same storage as a flat uint8 tensor (a contiguous halo region)."""
    import torch
    if t.dtype == torch.uint8:
        return t
    if not t.is_contiguous():
        raise ValueError("halo buffers must be contiguous")
    return t.reshape(-1).view(torch.uint8)


class HaloRing:
    """Per-rank halo state and the per-step protocol.

    halo:      the halo region directly in front of the segment (read by the head)
    tail:      the segment's last halo-length samples (sent to the next rank)
    incoming:  rank 0 only (G > 1): receive buffer for the next step's halo
    stage:     move the halo through host memory (a backend such as gloo that cannot send device
               tensors, e.g. several ranks sharing one GPU in tests); RCCL sends device tensors
               directly
    """

    def __init__(self, geom, halo, tail, incoming=None, stage: bool = False):
        self.geom, self.halo, self.tail, self.incoming = geom, halo, tail, incoming
        if geom.world > 1 and geom.rank == 0 and incoming is None:
            raise ValueError("rank 0 needs a receive buffer for the next step's halo")
        self.stage = stage and getattr(tail, "is_cuda", False)
        if self.stage:
            import torch
            self._send = torch.empty(tail.shape, dtype=tail.dtype, pin_memory=True)
            self._recv = torch.empty(tail.shape, dtype=tail.dtype, pin_memory=True)

    def _exchange(self, dst):
        import torch.distributed as dist
        g = self.geom
        send, recv = self.tail, dst
        if self.stage:
            self._send.copy_(self.tail)  # synchronous: the tail is final once this returns
            send, recv = self._send, self._recv
        # byte views: the halo is opaque samples, and ProcessGroupNCCL's send/recv have no complex
        # datatype ("Unconvertible NCCL type" for complex64; its collectives view complex as real,
        # its point-to-point ops do not)
        send, recv = _bytes(send), _bytes(recv)
        return dist.batch_isend_irecv([dist.P2POp(dist.isend, send, g.next_rank),
                                       dist.P2POp(dist.irecv, recv, g.prev_rank)])

    def _finish(self, reqs, dst):
        for r in reqs:
            r.wait()
        if self.stage:
            dst.copy_(self._recv)

    def step(self, bulk, head):
        """One sharded step. `bulk()` / `head()` launch the FIR over the segment-only outputs
        and over the outputs that read the halo. Returns after everything is enqueued."""
        g = self.geom
        if g.world == 1:
            bulk()
            head()
            self.halo.copy_(self.tail)  # history carry for the next step
            return
        dst = self.incoming if g.rank == 0 else self.halo
        reqs = self._exchange(dst)
        bulk()
        if g.rank == 0:
            head()  # halo arrived during the previous step
            self._finish(reqs, dst)
            self.halo.copy_(self.incoming)
        else:
            self._finish(reqs, dst)
            head()


class AmChainShard:
    """One rank's state for the time-sharded AM receive chain (ChainShardGeometry) on the GPU:
    buffer [halo | segment] of int8 IQ. One rank: the whole chain - RF FIR + AM + audio FIR - is ONE
    launch (gsdrInt8FirFCAmDemodFirFF, the AM samples never leave the chip). Several ranks: the bulk
    launch (segment-only RF windows and the audio outputs over them, fused; it runs while the halo
    exchange is in flight) and the head (RF windows reaching into the halo, then the first audio
    outputs, which read those AM samples). Weak scaling: every rank processes seg_len samples per step."""

    def __init__(self, geom: ChainShardGeometry, rf_taps, audio_taps, device, stage: bool = False, buf=None):
        """`buf`: an int8 view of 2 (halo + seg_len) bytes to work in (default: a fresh buffer). Views
        of one ring laid out segment after segment let a single rank read its history in place: the
        next view's halo IS this view's segment tail (step(carry=False))."""
        import torch
        self.geom, self.rf_taps, self.audio_taps = geom, rf_taps, audio_taps
        H, L = geom.halo, geom.seg_len
        if buf is None:
            buf = torch.zeros(2 * (H + L), dtype=torch.int8, device=device)
        if buf.dtype != torch.int8 or buf.numel() != 2 * (H + L):
            raise ValueError(f"AmChainShard: buf must be int8 with {2 * (H + L)} elements")
        self.buf = buf
        self.seg = self.buf[2 * H:]
        incoming = (torch.zeros(2 * H, dtype=torch.int8, device=device)
                    if geom.world > 1 and geom.rank == 0 else None)
        self.ring = HaloRing(geom, self.buf[: 2 * H], self.seg[2 * (L - H):], incoming, stage)
        self.am = torch.empty(geom.rf_outputs, dtype=torch.float32, device=device)
        self.out = torch.empty(geom.outputs, dtype=torch.float32, device=device)

    @property
    def head_audio(self) -> int:
        """Audio outputs whose window reaches into the head's AM samples [0, head_rf): j Da < head_rf
        (head_rf = halo / D is a multiple of Da by the halo's rounding)."""
        g = self.geom
        return min(g.outputs, -(-g.head_rf // g.audio_decimation))

    def _bulk(self):
        """RF outputs [head_rf, rf_outputs) and, in the same launch, the audio outputs whose windows
        lie in them (gsdrInt8FirFCAmDemodFirFF); the AM samples are kept for the head's audio.
        (r05 ran this launch and the head's on the 8-way kernel around a multi-rank fault of the 4-way
        one; r06 found the cause - window loads landing in registers the compiler had already reused,
        DESIGN.md 9 - and both run on the default kernel again.)"""
        from . import ops
        g = self.geom
        n_bulk = g.rf_outputs - g.head_rf
        ha = self.head_audio
        ops.am_chain_fused(self.rf_taps, self.seg, g.decimation, n_bulk, self.am[g.head_rf:], 0, self.audio_taps,
                           g.audio_decimation, g.outputs - ha, self.out[ha:], store_am=True)

    def _head(self):
        """RF outputs [0, head_rf) (they read the halo), then the audio outputs that read them."""
        from . import ops
        g = self.geom
        ops.fir(self.rf_taps, self.buf, g.decimation, g.head_rf, out=self.am[: g.head_rf], am=True, int8_iq=True)
        ha = self.head_audio
        if ha > 0:
            ops.fir(self.audio_taps, self.am, g.audio_decimation, ha, out=self.out[:ha])

    def step(self, carry_to=None, carry: bool = True):
        """One step over the segment currently in self.seg; the audio lands in self.out. A single
        rank (the halo is its own history) runs the RF stage as ONE launch over [halo | segment]
        (the halo is a multiple of D: the same outputs as the bulk and head launches) and copies the
        segment's tail to `carry_to` (default: its own halo), the next step's history - unless
        `carry` is False because the next step's halo already aliases the tail (ring views)."""
        from . import ops
        g = self.geom
        if g.world == 1:
            # ONE launch: RF FIR + AM + the audio FIR (the AM samples stay on chip, not stored)
            ops.am_chain_fused(self.rf_taps, self.buf, g.decimation, g.rf_outputs, self.am, 0, self.audio_taps,
                               g.audio_decimation, g.outputs, self.out, store_am=False)
            if carry:
                (self.ring.halo if carry_to is None else carry_to).copy_(self.ring.tail)
        else:
            self.ring.step(self._bulk, self._head)
        return self.out
