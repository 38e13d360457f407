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


class HaloRing:
    """Per-rank halo state and the per-step protocol.

    halo:      the (T-1)-sample region directly in front of the segment (read by the head)
    tail:      the segment's last T-1 samples (sent to the next rank)
    incoming:  rank 0 only (G > 1): receive buffer for the next step's halo
    """

    def __init__(self, geom: ShardGeometry, halo, tail, incoming=None):
        self.geom, self.halo, self.tail, self.incoming = geom, halo, tail, incoming
        if geom.world > 1 and geom.rank == 0 and incoming is None:
            raise ValueError("rank 0 needs a receive buffer for the next step's halo")

    def step(self, bulk, head):
        """One sharded step. `bulk()` / `head()` launch the FIR over the segment-only outputs
        and over the outputs that read the halo. Returns after everything is enqueued."""
        g = self.geom
        if g.world == 1:
            bulk()
            head()
            self.halo.copy_(self.tail)  # history carry for the next step
            return
        import torch.distributed as dist
        dst = self.incoming if g.rank == 0 else self.halo
        reqs = dist.batch_isend_irecv([dist.P2POp(dist.isend, self.tail, g.next_rank),
                                       dist.P2POp(dist.irecv, dst, g.prev_rank)])
        bulk()
        if g.rank == 0:
            head()  # halo arrived during the previous step
            for r in reqs:
                r.wait()
            self.halo.copy_(self.incoming)
        else:
            for r in reqs:
                r.wait()
            head()
