#!/usr/bin/env python3
"""Benchmark: Msamples/s through the FIR -> QuadAmDemod chain on MI355X (BASELINE.json metric).

Default workload (--workload c3, the north-star config): 2^28 - 6 cf32 samples per GPU step ->
1023-tap real-tap (FC) FIR, D = 10 -> QuadAmDemod, inputs resident in HBM. The FIR+AM runs as
gsdrFirFCAmDemod, which takes the polyphase overlap-save FFT kernel (fir_fft.hip) at this shape.
One GPU: the step is ONE launch over [T-1 history | segment]; the input / output buffer sets
rotate so that a step's working set is never resident in the 256 MiB Infinity Cache.

Multi-GPU (one process per GPU, torch.distributed over RCCL; `--gpus N` without a launcher
spawns the N ranks itself): the stream is time-sharded (gpusdr/shard.py). In step s rank g owns
samples [(s G + g) L, (s G + g + 1) L) and needs the preceding T - 1 samples, which live on rank
g - 1 (rank 0: rank G - 1's segment of the previous step): one ring exchange per step, overlapped
with the bulk launch that needs no halo; a head launch finishes the outputs that read the halo.
`--backend gloo --share-gpu` runs the same protocol with the ranks on one GPU (halos staged
through host memory), for testing.

Other workloads: c2 (BASELINE configs[1]: HackRF int8 IQ at 20 Msps, 127 taps, D = 1, the fused
gsdrInt8FirFCAmDemodCarry on the int8 MFMA kernel), c4 (cf32, 1023 taps, D = 1), c5 (the full AM
receive chain int8 IQ -> 1023-tap FIR, D = 10 -> AM -> 255-tap audio FIR, D = 20, 125 M samples
per GPU step; default `--c5-mode sharded`: time-sharded with the cascaded halo (Ta-1) D + T-1,
rounded to 3 600 samples; `resident` / `chunked`: the gsdrAmChain executor over one resident
segment, as one graph / as 25 chunk steps of 5 M samples in one cached graph).

Output: one JSON line on rank 0 (contract in the task statement) with `roofline` for the
dominant kernel (HIP events on its stream; `traffic` from the committed rocprofv3 PMC summary
profiles/pmc_traffic.json), `arithmetic` naming the kernel's number format, and `cpu_baseline`
(the oracle's float32 direct form on the host's cores, rank 0, N = 1, with the C1 config as a
second CPU line).
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "cuda-sdr_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "Msamples/sec through FIR→QuadAmDemod chain at 1/2/4/8 MI355X; % HBM roofline"
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md, spec
FP32_PEAK_TFLOPS = 157.3       # MI355X_MICROARCH.md, FP32 vector (packed FMA)
F16_PEAK_TFLOPS = 2500.0       # MI355X_MICROARCH.md, BF16/F16 MFMA dense

WORKLOADS = {
    # name: (description, input kind, samples per GPU step, taps, decimation, cutoff, window, fs)
    "c2": ("C2: HackRF int8 IQ @20 Msps -> cf32 -> 127-tap FC FIR -> QuadAmDemod, 1 s per GPU step",
           "i8", 20_000_000, 127, 1, 0.1, "hamming", 20e6),
    "c3": ("C3: wideband cf32 @200 Msps, 2^28 - 6 samples (a multiple of D) -> 1023-tap FC FIR, D=10 -> QuadAmDemod",
           "c64", (1 << 28) - (1 << 28) % 10, 1023, 10, 0.04, "blackman", 200e6),
    "c4": ("C4: cf32 stream, 1023-tap FC FIR, D=1 -> QuadAmDemod, 2^26 samples per GPU step",
           "c64", 1 << 26, 1023, 1, 0.04, "blackman", 1e9),
    "c4s": ("C4 (strong scaling): one 2^30-sample cf32 stream per step, 1023-tap FC FIR, D=1 -> QuadAmDemod, "
            "time-sharded over the N GPUs (2^30 / N samples per GPU step)",
            "c64", 1 << 30, 1023, 1, 0.04, "blackman", 1e9),
    "c5": ("C5: full AM chain @1 Gsps (1/8 per GPU): int8 IQ -> 1023-tap FC FIR, D=10 -> AM -> 255-tap FF "
           "FIR, D=20, 125 M samples (1 s) per GPU step",
           "i8", 125_000_000, 1023, 10, 0.04, "blackman", 1e9),
}
STRONG = {"c4s"}  # workloads whose samples per step are the WHOLE job's, split over the ranks
C5_CHUNK = 5_000_000   # multiple of D * Da = 200
C5_AUDIO = (255, 20, 0.02, "hamming")


def lowpass(num_taps, cutoff, window):
    n = np.arange(num_taps, dtype=np.float64) - (num_taps - 1) / 2.0
    h = 2.0 * cutoff * np.sinc(2.0 * cutoff * n)
    m = np.arange(num_taps, dtype=np.float64)
    if window == "hamming":
        w = 0.54 - 0.46 * np.cos(2 * np.pi * m / (num_taps - 1))
    else:
        w = 0.42 - 0.5 * np.cos(2 * np.pi * m / (num_taps - 1)) + 0.08 * np.cos(4 * np.pi * m / (num_taps - 1))
    h = h * w
    return (h / h.sum()).astype(np.float32)


def dist_setup(n_gpus, backend="nccl", share_gpu=False):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n_gpus:
        raise SystemExit(f"bench.py: --gpus {n_gpus} but WORLD_SIZE={world}; launch one rank per GPU "
                         "(torch.distributed.run) or let bench.py spawn them (WORLD_SIZE unset)")
    dev_index = 0 if share_gpu else local
    torch.cuda.set_device(dev_index)
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev_index))
        else:
            dist.init_process_group(backend)
    return rank, world, dev_index


# Each step streams at least this many bytes through distinct buffers, so a step's working set never
# sits in the 256 MiB Infinity Cache (MI355X_MICROARCH.md: FETCH_SIZE counts MALL hits; C2's one
# second of signal is only 120 MB): the input / output buffer sets rotate step by step.
MALL_BYTES = 256 << 20


class _Slot:
    """One [halo | segment] input buffer, its output, and its halo ring."""

    def __init__(self, g, w, dt, device, ring_cls, stage, incoming, buf=None):
        H, L = g.halo, g.seg_len
        self.buf = torch.zeros(w * (H + L), dtype=dt, device=device) if buf is None else buf
        self.seg = self.buf[w * H:]
        self.ring = ring_cls(g, self.buf[: w * H], self.seg[w * (L - H):], incoming, stage)
        self.bulk_x = self.seg[w * g.bulk_input_offset():]
        self.out = torch.empty(g.outputs, dtype=torch.float32, device=device)


class ShardedChain:
    """Per-rank state of one time-sharded FIR -> AM step (gpusdr/shard.py protocol)."""

    def __init__(self, ops, wl, rank, world, device, stage=False):
        from gpusdr.shard import HaloRing, ShardGeometry
        desc, kind, L, T, D, cutoff, window, fs = WORKLOADS[wl]
        if wl in STRONG:  # the job's fixed stream per step, split over the ranks
            L = L // world // D * D
        self.ops, self.kind, self.L, self.T, self.D = ops, kind, L, T, D
        self.geom = g = ShardGeometry(rank, world, L, T, D)
        H = g.halo
        self.taps = torch.from_numpy(lowpass(T, cutoff, window)).to(device)
        w = 2 if kind == "i8" else 1  # tensor elements per sample (int8 I,Q | complex64)
        dt = torch.int8 if kind == "i8" else torch.complex64
        step_bytes = (H + L) * (2 if kind == "i8" else 8) + g.outputs * 4
        self.n_slots = max(1, -(-int(1.5 * MALL_BYTES) // step_bytes))
        incoming = torch.zeros(w * H, dtype=dt, device=device) if (world > 1 and rank == 0) else None
        # one rank: the slots are consecutive views of one input ring when 4 of them fit 20 GB, so
        # slot k + 1's halo IS slot k's segment tail and only the wrap copies the history (as a live
        # receiver's input ring holds it; 2^28 cf32 samples: one 8 KB copy per 4 steps, not per step)
        self.ring = world == 1 and 4 * step_bytes <= 20 * 2**30
        if self.ring:
            self.n_slots = max(self.n_slots, 4)
            ring = torch.zeros(w * (H + self.n_slots * L), dtype=dt, device=device)
            self.slots = [_Slot(g, w, dt, device, HaloRing, stage, incoming, buf=ring[w * k * L: w * (k * L + H + L)])
                          for k in range(self.n_slots)]
        else:
            self.slots = [_Slot(g, w, dt, device, HaloRing, stage, incoming) for _ in range(self.n_slots)]
        for k, sl in enumerate(self.slots):  # slot k holds the stream position of step k
            if kind == "i8":
                ops.synth_iq_int8(0x5EED, fs, 1e3, fs * 0.075, g.segment_start(k), L, out=sl.seg)
            else:
                ops.synth_wideband_cf32(0xC3, 0.013, 0.31, g.segment_start(k), L, out=sl.seg)
        self.cur = 0
        self.ev = None
        if world == 1:  # the step's launch per slot, validated once (a C2 launch is ~36 us: the
            # argument checks of ops.fir on every step would leave the GPU waiting for the host)
            for sl in self.slots:
                sl.launch = ops.bind_fir(self.taps, sl.buf, D, g.outputs, sl.out, am=True, int8_iq=(kind == "i8"))

    @property
    def slot(self):
        return self.slots[self.cur]

    @property
    def buf(self):
        return self.slot.buf

    def _fir(self, x, n_out, out):
        if n_out > 0:
            self.ops.fir(self.taps, x, self.D, n_out, out=out, am=True, int8_iq=(self.kind == "i8"))

    @property
    def single(self):
        """World 1: the whole step is ONE launch over [history | segment]; for int8 IQ the
        history carry for the next step is fused into it (gsdrInt8FirFCAmDemodCarry)."""
        return self.geom.world == 1

    def bulk(self):
        """Outputs [head, L/D): inputs entirely inside this rank's segment (the timed kernel)."""
        g, sl = self.geom, self.slot
        if self.ev is not None:
            self.ev[0].record()
        self._fir(sl.bulk_x, g.outputs - g.head_outputs, sl.out[g.head_outputs:])
        if self.ev is not None:
            self.ev[1].record()

    def head(self):
        """Outputs [0, head): read the halo in front of the segment."""
        sl = self.slot
        self._fir(sl.buf, self.geom.head_outputs, sl.out[: self.geom.head_outputs])

    def step(self, ev=None):
        self.ev = ev
        g, sl = self.geom, self.slot
        nxt = self.slots[(self.cur + 1) % self.n_slots]
        if not self.single:
            sl.ring.step(self.bulk, self.head)
            if self.n_slots > 1 and g.rank == 0:
                nxt.ring.halo.copy_(sl.ring.halo)  # the halo that arrived for the next step
        else:
            if ev is not None:
                ev[0].record()
            # ring views: the next slot's halo already holds this segment's tail (except at the wrap)
            in_place = self.ring and self.cur != self.n_slots - 1
            fused_carry = self.kind == "i8" and self.D == 1 and not in_place
            # the fused carry writes the unconsumed tail (T - D samples); with D = 1 that is the
            # whole T - 1 halo in front of the next step's segment
            if fused_carry:
                self.ops.fir_am_i8_carry(self.taps, sl.buf, self.D, g.outputs, sl.out, nxt.ring.halo)
            else:
                sl.launch()
            if ev is not None:
                ev[1].record()
            if not in_place and not fused_carry:
                nxt.ring.halo.copy_(sl.ring.tail)
        self.cur = (self.cur + 1) % self.n_slots

    @property
    def kernel_class(self):
        x = self.slot.buf if self.single else self.slot.bulk_x
        return self.ops.fir_kernel_class(x, self.taps, self.D, int8_iq=(self.kind == "i8"))

    def timed_bytes_ops(self):
        """Algorithmic bytes of the timed launch (input read once + output written once) and the
        arithmetic the kernel performs: (kind, flops, peak TFLOP/s of the unit it runs on)."""
        g = self.geom
        n = g.outputs if self.single else g.outputs - g.head_outputs
        n_in = (n - 1) * self.D + self.T
        in_bytes = n_in * (2 if self.kind == "i8" else 8)
        return in_bytes + n * 4, kernel_compute(self.kernel_class, n, self.T, self.D)


class AmChainSharded:
    """C5 default: the time-sharded AM receive chain (gpusdr.shard.AmChainShard) - every rank runs
    int8 IQ -> 1023-tap FIR, D = 10 -> AM -> 255-tap audio FIR, D = 20 over [cascaded halo |
    segment], the halo ((Ta - 1) D + T - 1 -> 3 600 samples) coming from the previous rank over the
    ring (its own previous step at N = 1). Input slots rotate past the Infinity Cache."""

    def __init__(self, ops, rank, world, device, stage=False):
        from gpusdr.shard import AmChainShard, ChainShardGeometry
        desc, kind, L, T, D, cutoff, window, fs = WORKLOADS["c5"]
        Ta, Da, cut_a, win_a = C5_AUDIO
        self.ops, self.kind, self.L, self.T, self.D, self.Ta, self.Da = ops, kind, L, T, D, Ta, Da
        self.mode = "sharded"
        self.geom = g = ChainShardGeometry(rank, world, L, T, D, Ta, Da)
        rf = torch.from_numpy(lowpass(T, cutoff, window)).to(device)
        au = torch.from_numpy(lowpass(Ta, cut_a, win_a)).to(device)
        self.rf_taps = rf
        step_bytes = 2 * (g.halo + L) + 4 * g.rf_outputs + 4 * g.outputs
        self.n_slots = max(1, -(-int(1.5 * MALL_BYTES) // step_bytes))
        self.single = world == 1
        if self.single:
            # one rank: the slots are consecutive views of one input ring, so slot k + 1's halo IS slot
            # k's segment tail (a live receiver's ring holds its history in front of the new samples);
            # only the wrap back to slot 0 copies the history. 8 slots: one 7 KB copy per 8 steps.
            self.n_slots = max(self.n_slots, 8)
            ring = torch.zeros(2 * (g.halo + self.n_slots * L), dtype=torch.int8, device=device)
            self.slots = [AmChainShard(g, rf, au, device, stage, buf=ring[2 * k * L: 2 * (k * L + g.halo + L)])
                          for k in range(self.n_slots)]
        else:
            self.slots = [AmChainShard(g, rf, au, device, stage) for _ in range(self.n_slots)]
        for k, sh in enumerate(self.slots):
            ops.synth_iq_int8(0x5EED, fs, 1e3, fs * 0.075, g.segment_start(k), L, out=sh.seg)
        self.cur = 0
        self.kernel_class = ops.fir_kernel_class(self.slots[0].seg, rf, D, int8_iq=True)

    def step(self, ev=None):
        g, sh = self.geom, self.slots[self.cur]
        nxt = self.slots[(self.cur + 1) % self.n_slots]
        if ev is not None:
            ev[0].record()
        # one rank: the next slot's halo already holds this segment's tail, except at the wrap
        if g.world == 1:
            last = self.cur == self.n_slots - 1
            sh.step(carry_to=nxt.ring.halo, carry=last)
        else:
            sh.step()
        if ev is not None:
            ev[1].record()
        if self.n_slots > 1 and g.world > 1 and g.rank == 0:
            nxt.ring.halo.copy_(sh.ring.halo)
        self.cur = (self.cur + 1) % self.n_slots

    def timed_bytes_ops(self):
        """Per step (the timed region is the whole step: RF FIR + AM bulk and head, audio FIR):
        int8 input (segment + halo) read once + audio written once; RF kernel arithmetic plus the
        audio FIR's direct-form flops."""
        g = self.geom
        kind, fl, peak = kernel_compute(self.kernel_class, g.rf_outputs, self.T, self.D)
        return 2 * (g.halo + self.L) + 4 * g.outputs, (f"RF: {kind}; audio FIR: fp32 VALU on the RF kernel's "
                                                       "producer waves (N = 1) / direct form",
                                                       fl + g.outputs * self.Ta * 2, peak)


def kernel_compute(cls, n_out, T, D):
    """(kind, flops per launch, peak TFLOP/s) of the FIR kernel family `cls` for n_out outputs."""
    if cls == "fft":
        fft = 5 * 512 * 9  # nominal 5 N log2 N per 512-point FFT
        kind = "fp32 FFT fast convolution (polyphase overlap-save, 512-point FFTs; nominal 5 N log2 N)"
        if D == 1:  # firFftD1PfKernel: 8 input-phase FFTs, the phase stage (per frequency 22 complex
            # products and two 8-point DFTs, nominal 5 N log2 N), 8 inverse FFTs per block
            V = 512 - -(-T // 8)
            blocks = -(-n_out // (8 * V))
            return kind, blocks * (8 * fft + 512 * (22 * 6 + 2 * 5 * 8 * 3) + 8 * fft), FP32_PEAK_TFLOPS
        Q = -(-T // D)
        V = 512 - Q + 1
        blocks = -(-n_out // V)
        return kind, blocks * (D * fft + D * 512 * 8 + fft), FP32_PEAK_TFLOPS
    if cls == "i8-mfma":
        s = (T + 62) // 32  # K-blocks of 32: K = 32 S >= T + 31
        return ("f16 MFMA (2 tap limbs, fp32 accumulate)", n_out * 2 * 2 * 32 * s * 2, F16_PEAK_TFLOPS)
    if cls == "i8-dec-mfma":
        # the 4-way kernel (fir_i8_ws4.hip, r05): the smallest instantiated K quarter of 16-wide steps that
        # covers 31 D + T (kW4KS); the 8-way one (firI8WsKernel: GSDR_POLICY_I8_WS8, or no 4-way KS
        # fits): 8 waves x ceil(K-steps / 8). Two f16 tap limbs, fp32 accumulate.
        ksteps = -(-(31 * D + T) // 16)
        need = -(-ksteps // 4)
        fits = [k for k in (2, 4, 6, 8, 11, 14, 17, 21, 22) if k >= need]
        if i8_ws8_policy() or not fits:
            k_pad = 8 * 16 * -(-ksteps // 8)
        else:
            k_pad = 4 * 16 * min(fits)
        return (f"f16 MFMA (split precision, 2 products, padded Toeplitz K = {k_pad}, fp32 accumulate)",
                n_out * 2 * k_pad * 2 * 2, F16_PEAK_TFLOPS)
    if cls == "cf-mfma":
        ksteps = -(-(31 * D + T) // 16)  # Toeplitz K in steps of 16; 8 consumer waves, KS K-steps each
        k_pad = 8 * 16 * -(-ksteps // 8)
        return (f"f16 MFMA (split precision, 3 products, padded Toeplitz K = {k_pad}, fp32 accumulate)",
                n_out * 2 * k_pad * 3 * 2, F16_PEAK_TFLOPS)
    return ("fp32 VALU FMA (direct form)", n_out * T * 4, FP32_PEAK_TFLOPS)


class AmChainRunner:
    """C5: the gsdrAmChain executor (one hipGraph per chunk) over a resident 1-second segment.

    Each rank owns its own time range of the synthetic 1 Gsps stream (rank g starts at g * L);
    the chain history carries across steps, and the warm-up steps prime it, so the timed steps are
    all steady-state (no data-path collective; weak scaling)."""

    def __init__(self, ops, rank, world, device, mode="resident"):
        from gpusdr.chain import AmChain
        desc, kind, L, T, D, cutoff, window, fs = WORKLOADS["c5"]
        Ta, Da, cut_a, win_a = C5_AUDIO
        self.kind, self.L, self.T, self.D, self.Ta, self.Da = kind, L, T, D, Ta, Da
        self.mode = mode
        self.chunks = L // C5_CHUNK
        assert self.chunks * C5_CHUNK == L
        self.chain = AmChain(lowpass(T, cutoff, window), D, lowpass(Ta, cut_a, win_a), Da, C5_CHUNK, device.index)
        # [RF history | 1 s segment]: resident steps read the history in place in front of it
        self.hist = 2 * 2048
        self.buf = torch.empty(self.hist + 2 * L, dtype=torch.int8, device=device)
        ops.synth_iq_int8(0x5EED, fs, 1e3, fs * 0.075, rank * L, L + self.hist // 2, out=self.buf)
        self.iq = self.buf[self.hist:]
        self.out = torch.empty(L // (D * Da) + C5_CHUNK, dtype=torch.float32, device=device)
        self.stream = self.chain.torch_stream
        self.geom = None
        self.single = world == 1
        self.kernel_class = ops.fir_kernel_class(self.iq, torch.from_numpy(lowpass(T, cutoff, window)), D,
                                                 int8_iq=True)

    def step(self, ev=None):
        with torch.cuda.stream(self.stream):
            if ev is not None:
                ev[0].record(self.stream)
            if self.mode == "resident":
                self.chain.step_resident(self.iq, self.chunks, self.out)
            else:  # live-stream chunks, all of a step's chunk steps as one cached graph launch
                self.chain.step_chunks(self.iq, self.chunks, self.out)
            if ev is not None:
                ev[1].record(self.stream)

    def timed_bytes_ops(self):
        """Per timed region (all chunks of a step): int8 input read once + audio written once; the
        RF FIR kernel's arithmetic plus the audio FIR's direct-form flops (2 Ta / Da per AM sample)."""
        n_rf = self.L // self.D
        n_audio = n_rf // self.Da
        kind, fl, peak = kernel_compute(self.kernel_class, n_rf, self.T, self.D)
        return 2 * self.L + 4 * n_audio, (f"RF: {kind}; audio FIR: fp32 VALU direct form", fl + n_audio * self.Ta * 2,
                                          peak)


def cpu_threads():
    """Host threads for the CPU baseline: every core this process may run on, capped at the
    job's CPU share when the launcher states one (OMP_NUM_THREADS; 16 per GPU on the GPU box,
    whose os.cpu_count() reports the whole machine)."""
    avail = len(os.sched_getaffinity(0))
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        return min(avail, int(share)), avail
    return avail, avail


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_c1(oracle, threads):
    """C1 (BASELINE.json configs[0]) in full: CosineSource(fs=1e6, f=12345 Hz) -> 63-tap FF FIR,
    1 M f32 samples, float32 direct form on the host cores (median of 10 after 2 warm-ups)."""
    n = 1 << 20
    delta = float(np.float32(2.0 * np.pi * 12345.0 / 1e6))
    x = oracle.cosine_f(0.0, float(np.float32(n * delta)), n)
    taps = oracle.lowpass_taps(63, 0.1)
    n_out = oracle.fir_output_count(n, 63, 1)
    for _ in range(2):
        oracle.fir_ff_f32(taps, x, 1, n_out, threads, baseline=True)
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        oracle.fir_ff_f32(taps, x, 1, n_out, threads, baseline=True)
        ts.append(time.perf_counter() - t0)
    dt = float(np.median(ts))
    return {"config": "C1: CosineSource f32 (fs 1e6, 12345 Hz) -> 63-tap FF FIR, 1,048,576 samples, D=1",
            "value": n / dt / 1e6, "unit": "Msamples/s", "ms": dt * 1e3, "cores": threads}


def cpu_baseline(wl, seconds_target=8.0):
    """Oracle port (float32 direct form, the host cores) on a bounded sample of workload `wl`,
    plus the C1 CPU configuration run in full."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle  # noqa: E402  (cpu_baseline leg only)
    desc, kind, L, T, D, cutoff, window, fs = WORKLOADS[wl]
    taps = lowpass(T, cutoff, window)
    threads, avail = cpu_threads()
    n_out = 1 << 16
    while True:
        n_in = (n_out - 1) * D + T
        if kind == "i8":
            x = oracle.synth_iq_int8(0x5EED, fs, 1e3, fs * 0.075, 0, n_in)
            run = lambda: oracle.chain_i8_fc_am_f32(taps, x, D, n_out, threads, baseline=True)  # noqa: E731
        else:
            x = oracle.synth_wideband_cf32(0xC3, 0.013, 0.31, 0, n_in)
            run = lambda: oracle.chain_fc_am_f32(taps, x, D, n_out, threads, baseline=True)  # noqa: E731
        run()  # warm
        t0 = time.perf_counter()
        run()
        dt = time.perf_counter() - t0
        if dt >= seconds_target / 4 or n_out >= (1 << 26):
            break
        n_out = int(n_out * min(16.0, max(2.0, (seconds_target / 4) / max(dt, 1e-4))))
    reps = max(1, int(seconds_target / max(dt, 1e-3)))
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    dt = (time.perf_counter() - t0) / reps
    return {
        "value": (n_out * D) / dt / 1e6,
        "unit": "Msamples/s",
        "cores": threads,
        # per core, so the all-cores figure of north_star extrapolates (the job gets a CPU share)
        "per_core_msps": (n_out * D) / dt / 1e6 / threads,
        "host_cpus": os.cpu_count(),
        "affinity_cpus": avail,
        "cpu_model": _cpu_model(),
        "isa": oracle.baseline_isa(),
        "kind": "port",
        "sample": f"{n_out * D} input samples of the {wl} chain (oracle/gsdr_oracle.c float32 direct form, "
                  f"{threads} threads = {'the job CPU share (OMP_NUM_THREADS)' if threads < avail else 'all cores'}"
                  f" of {avail} schedulable, mean of {reps} runs"
                  + ("; RF FIR + AM only, the audio FIR is 0.6 % of the flops)" if wl == "c5" else ")"),
        "c1": cpu_c1(oracle, threads),
    }


KERNEL_POLICY = 0  # --kernel-policy (gsdrAmdSetKernelPolicy flags) of this run


def i8_ws8_policy():
    """The int8 decimating launches run on the 8-way kernel (GSDR_POLICY_I8_WS8 = 64)."""
    return bool(KERNEL_POLICY & 64)


def i8_dec_kernel(T, D):
    """The wave-specialised int8 kernel a decimating launch of (T, D) runs on."""
    need = -(-(-(-(31 * D + T) // 16)) // 4)
    return "firI8WsKernel" if i8_ws8_policy() or need > 22 else "firI8Ws4Kernel"


def kernel_name(chain):
    if isinstance(chain, AmChainSharded):
        body = {"fft": "firFftKernel", "i8-dec-mfma": i8_dec_kernel(chain.T, chain.D), "valu": "firLdsKernel"}.get(
            chain.kernel_class, chain.kernel_class)
        if chain.single:
            return (f"whole C5 step: gsdrInt8FirFCAmDemodFirFF ({body}<.., AUD>: RF FIR + AM + audio FIR in one "
                    "launch); HIP events around the step")
        return (f"whole C5 step: gsdrInt8FirFCAmDemodFirFF bulk ({body}<.., AUD>), then the head: "
                "gsdrInt8FirFCAmDemod + gsdrFirFF over the head's audio windows; HIP events around the step")
    if isinstance(chain, AmChainRunner):
        return (f"gsdrAmChain {chain.mode} step graph (RF FIR+AM+audio FIR fused per launch, history copies; "
                "HIP events around the whole step)")
    entry = ("gsdrInt8FirFCAmDemodCarry" if chain.single else "gsdrInt8FirFCAmDemod") if chain.kind == "i8" \
        else "gsdrFirFCAmDemod"
    body = {"fft": "firFftD1PfKernel" if chain.D == 1 else "firFftKernel", "i8-mfma": "firI8MfmaKernel",
            "i8-dec-mfma": i8_dec_kernel(chain.T, chain.D), "cf-mfma": "firCfWsKernel",
            "valu": "firLdsKernel"}[chain.kernel_class]
    return f"{entry} ({body})"


def load_traffic(wl):
    """(HBM bytes per launch, where that figure was measured) of the dominant kernel from the
    committed rocprofv3 PMC summary profiles/pmc_traffic.json."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            e = json.load(f).get(wl, {})
        return e.get("hbm_bytes_per_launch"), ({"kernel": e.get("kernel"), "launches": e.get("launches"),
                                                "note": e.get("note")} if e else None)
    except (OSError, ValueError):
        return None, None


def _free_port():
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _spawned_rank(local_rank, argv, world, port):
    """Child of spawn_ranks: a fresh interpreter per GPU (nothing touched the GPU in the parent)."""
    os.environ.update({"RANK": str(local_rank), "LOCAL_RANK": str(local_rank), "WORLD_SIZE": str(world),
                       "LOCAL_WORLD_SIZE": str(world), "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    sys.argv = [sys.argv[0]] + list(argv)
    main()


def spawn_ranks(n, share_gpu=False):
    """`bench.py --gpus N` without a launcher: start N fresh rank processes (spawn, so no process
    inherits a GPU context) and wait for them; the parent never initialises the GPU."""
    import torch.multiprocessing as mp
    have = torch.cuda.device_count()  # does not initialise the GPU on this image
    if have < n and not share_gpu:
        raise SystemExit(f"bench.py: --gpus {n} but only {have} GPU(s) visible "
                         "(--share-gpu --backend gloo runs the ranks on one GPU, for testing)")
    mp.start_processes(_spawned_rank, args=(sys.argv[1:], n, _free_port()), nprocs=n, join=True,
                       start_method="spawn")


SETTLE_S = 0.25  # untimed settle before the warm-up steps (see settle)


def settle(step, seconds=SETTLE_S, world=1, device=None, backend="nccl"):
    """Run `step` untimed for ~`seconds`: after idle the GPU needs ~10-20 ms of load to leave its
    low-clock power state - the first ~20-30 C3 launches take 0.66 ms instead of 0.48 ms
    (profiles/r03/exp/c3_bench_loop_probe.log) - so 5 warm-up steps alone left the timed steps in
    the ramp. Nothing timed is skipped: the K timed steps still do the full work.
    With several ranks every rank must run the SAME number of steps (each step exchanges halos
    with the ring neighbours; a rank one step short leaves its neighbour waiting for a halo that
    never comes - a 2-rank C5 run hung that way in r04): rank 0 times 8 steps, picks the count for
    `seconds` and broadcasts it."""
    if world == 1:
        t0 = time.perf_counter()
        n = 0
        while time.perf_counter() - t0 < seconds and n < 4096:
            step()
            n += 1
            if n % 8 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        return
    t0 = time.perf_counter()
    for _ in range(8):
        step()
    torch.cuda.synchronize()
    per = max((time.perf_counter() - t0) / 8, 1e-6)
    more = torch.tensor([max(0, min(4096, int(seconds / per)) - 8)], dtype=torch.int64,
                        device=device if backend == "nccl" else "cpu")
    dist.broadcast(more, 0)
    for i in range(int(more.item())):
        step()
        if (i + 1) % 8 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()


def timed_steps(chain, steps, warmup, world, backend, device, local, ops):
    """A short settle, W untimed warm-up steps, then K steps between barrier + synchronize on both
    sides; the max over ranks of the wall time, and the mean per-step HIP-event time of the timed
    kernel."""
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    # no Python garbage collection inside the timed region: a C2 step is ~40 us of GPU time, and one
    # collection pause of the objects the earlier workloads left (~10 ms) inflated a 50-step C2 line
    # 5x in an r04 default run (0.221 ms/step beside 0.036 ms launches). The collection runs BEFORE
    # the settle: run between the warm-up and the timed steps it idled the GPU for 45-62 ms, and the
    # power controller's answer to that idle (a few fast launches, then a clock dip recovering over
    # ~40 launches: C3 464 -> 725 -> 500 us, C5 183 -> 226 -> 190 us in one trace,
    # profiles/r04/exp/bench_idle_gap/) landed inside the timed region: C3 0.56-0.59 ms per step
    # against 0.48-0.49 ms of kernel time in the same run.
    ops.fft_direct_blocks(local, reset=True)  # first call outside the timed path (symbol lookup)
    gc.collect()
    gc.disable()
    try:
        if world > 1:
            # ranks start the settle together, so they also leave it together: a rank that waited
            # long at the barrier before the timed steps would start them after an idle gap
            dist.barrier()
        settle(chain.step, world=world, device=device, backend=backend)
        for _ in range(warmup):
            chain.step()
        ops.fft_direct_blocks(local, reset=True)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for i in range(steps):
            chain.step(evs[i])
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        elapsed = time.perf_counter() - t0
    finally:
        gc.enable()
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64, device=device if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    kernel_ms = float(np.mean([a.elapsed_time(b) for a, b in evs]))
    return elapsed, kernel_ms, ops.fft_direct_blocks(local, reset=True)


def extra_line(wl, chain, elapsed, kernel_ms, steps, world):
    """A secondary workload measured in the same run (same protocol as the headline)."""
    bytes_, (kind, fl, peak) = chain.timed_bytes_ops()
    gbs = bytes_ / (kernel_ms * 1e-3) / 1e9
    strong = wl in STRONG
    return {"workload": WORKLOADS[wl][0], "value": world * chain.L * steps / elapsed / 1e6, "unit": "Msamples/s",
            "n_gpus": world, "steps": steps, "ms_per_step": elapsed / steps * 1e3,
            "scaling": "strong" if strong else "weak", "samples_per_gpu_step": chain.L,
            "kernel": kernel_name(chain), "kernel_class": chain.kernel_class,
            "achieved_gbs": gbs, "frac": gbs / HBM_PEAK_GBS, "avg_launch_ms": kernel_ms,
            "algorithmic_bytes_per_launch": bytes_,
            # the unit the kernel computes on (C5's RF stage is MFMA-bound: its HBM frac is not its bound)
            "compute": {"kind": kind, "achieved_tflops": fl / (kernel_ms * 1e-3) / 1e12, "peak_tflops": peak,
                        "frac": fl / (kernel_ms * 1e-3) / 1e12 / peak, "flops_per_launch": fl,
                        "direct_form_flops_per_launch": direct_form_flops(wl, chain)}}


def direct_form_flops(wl, chain):
    """SURVEY 8(d) flop convention: direct-form counts (FC 4 T / D per input sample, FF 2 T / D), i.e.
    the useful work, against which a padded MFMA or an FFT count can be compared."""
    if wl == "c5":
        g = chain.geom
        n_rf = g.rf_outputs if g is not None else chain.L // chain.D
        return n_rf * 4 * chain.T + (n_rf // chain.Da) * 2 * chain.Ta
    g = chain.geom
    n = g.outputs if chain.single else g.outputs - g.head_outputs  # the timed launch's outputs
    return n * 4 * chain.T


def mixed_vs_plain(ops, chain, reps=10):
    """The fused frequency shifter on the C3 kernel: gsdrMixFirFCAmDemod (mixer folded into the FFT
    kernel: row chirp, c_p in G) against gsdrFirFCAmDemod over the same resident C3 input, HIP
    events around `reps` launches each (interleaved twice)."""
    x, n = chain.slot.buf, chain.geom.outputs
    out = torch.empty(n, dtype=torch.float32, device=x.device)
    ts = {"plain": [], "mixed": []}
    settle(lambda: ops.fir(chain.taps, x, chain.D, n, out=out, am=True), 0.1)
    for _ in range(2):
        for kind in ("plain", "mixed"):
            mix = (0.3, -2 * np.pi * 0.0731) if kind == "mixed" else None
            ops.fir(chain.taps, x, chain.D, n, out=out, am=True, mix=mix)
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(reps):
                ops.fir(chain.taps, x, chain.D, n, out=out, am=True, mix=mix)
            b.record()
            b.synchronize()
            ts[kind].append(a.elapsed_time(b) / reps)
    plain, mixed = min(ts["plain"]), min(ts["mixed"])
    return {"what": "C3 shape (2^28 - 6 cf32, 1023 taps, D = 10, AM): gsdrMixFirFCAmDemod vs gsdrFirFCAmDemod",
            "plain_ms": plain, "mixed_ms": mixed, "mixed_over_plain": mixed / plain}


def host_fed_c5(device, slots=4, warmup=8, steps=48):
    """C5 fed from host memory (north_star: src/buffers -> pinned hipHostMalloc ring buffers;
    the reference's ingest CudaMemcpyFilter.cpp:28-104): the gsdrAmChain executor with a ring of
    `slots` pinned input / output slots of one 5 M-sample chunk each; per step the chunk's H2D copy
    runs on the chain's second stream, overlapped with the previous steps' compute, and the audio
    returns into a pinned output slot. The input slots are filled once (synthetic IQ); every step
    still copies its 10 MB across PCIe. Reported beside `value` (PCIe-inclusive), never as it."""
    from gpusdr.chain import AmChain
    desc, kind, L, T, D, cutoff, window, fs = WORKLOADS["c5"]
    Ta, Da, cut_a, win_a = C5_AUDIO
    chain = AmChain(lowpass(T, cutoff, window), D, lowpass(Ta, cut_a, win_a), Da, C5_CHUNK, device.index,
                    host_slots=slots)
    from gpusdr import ops
    for s in range(slots):
        iq = ops.synth_iq_int8(0x5EED, fs, 1e3, fs * 0.075, s * C5_CHUNK, C5_CHUNK, device=device)
        chain.host_input(s)[:] = iq.cpu().numpy()
    counts = [0] * slots
    audio = 0

    def run(n, first):
        nonlocal audio
        for k in range(first, first + n):
            s = k % slots
            if k >= slots:  # the slot's previous step must be done before it is refilled / reused
                audio += len(chain.wait_host(s, counts[s]))
            counts[s] = chain.step_host(s)

    run(warmup, 0)
    torch.cuda.synchronize()
    audio = 0
    t0 = time.perf_counter()
    run(steps, warmup)
    for k in range(warmup + steps - slots, warmup + steps):
        audio += len(chain.wait_host(k % slots, counts[k % slots]))
    dt = time.perf_counter() - t0
    chain.close()
    msps = steps * C5_CHUNK / dt / 1e6
    # the link itself: pinned host -> device copies of one chunk's bytes on a side stream (the
    # ceiling this line can reach; PCIe Gen5 x16 is ~50 GB/s per direction where it is not shared)
    hb = torch.empty(2 * C5_CHUNK, dtype=torch.int8, pin_memory=True)
    db = torch.empty(2 * C5_CHUNK, dtype=torch.int8, device=device)
    cs = torch.cuda.Stream(device)
    with torch.cuda.stream(cs):
        for _ in range(3):
            db.copy_(hb, non_blocking=True)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(cs)
        for _ in range(20):
            db.copy_(hb, non_blocking=True)
        b.record(cs)
    b.synchronize()
    h2d_gbs = 20 * 2 * C5_CHUNK / (a.elapsed_time(b) * 1e-3) / 1e9
    del hb, db
    return {"workload": f"C5 fed from host memory: {slots} pinned hipHostMalloc slots of {C5_CHUNK} int8 IQ samples, "
                        "H2D on the chain's copy stream overlapped with compute, audio back into pinned slots",
            "value": msps, "unit": "Msamples/s", "steps": steps, "ms_per_step": dt / steps * 1e3,
            "h2d_gbs": msps * 2e6 / 1e9, "h2d_link_probe_gbs": h2d_gbs, "audio_samples": audio,
            "note": "PCIe-inclusive rate, reported beside value (inputs resident in HBM), never as it"}


def hbm_probe(ops, device, nbytes=2 << 30, reps=10):
    """Measured HBM bandwidth in this process (% of spec AND of measured copy BW):
    gsdrAmdHbmProbe streaming-read (float4 loads, one sum per thread) and copy kernels over `nbytes`
    buffers, HIP events around `reps` launches after two warm-ups; GB/s of bytes moved (copy:
    read + write)."""
    src = torch.empty(nbytes // 4, dtype=torch.float32, device=device).fill_(1.0)
    dst = torch.empty_like(src)
    res = {}
    for mode, name, moved in ((0, "read", nbytes), (1, "copy", 2 * nbytes)):
        for _ in range(2):
            ops.hbm_probe(src, dst, mode)
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(reps):
            ops.hbm_probe(src, dst, mode)
        b.record()
        b.synchronize()
        ms = a.elapsed_time(b) / reps
        res[name + "_gbs"] = moved / (ms * 1e-3) / 1e9
    del src, dst
    torch.cuda.empty_cache()
    res["bytes"] = nbytes
    return res


def node_path(ops, device, kernel_value, segments=11, warmup=1):
    """C3 through the reference's filter-graph API (getFactoriesSingleton nodes, SteppingDriver):
    Fir(real taps, FloatComplex, D = 10) -> QuadAmDemod -> a device sink taking one C3 segment of AM
    output per step. The Fir window is pre-filled with `segments` C3 segments (2^28 - 6 samples each,
    outside the timed region: an upstream node would write them there); each fused driver step then
    moves one segment (the device sink grows its window exactly to the request) in ONE
    gsdrFirFCAmDemod launch; unfused, the reference's Fir and QuadAmDemod launches with the cf32
    intermediate in the AM window, which the Fir may fill ahead by its headroom (outputs are counted
    from the windows, not assumed). Also the host time of one
    driver step, eager vs replayed (doFilterGraphed), on 1 MiB pushes (the reference's chunk)."""
    from gpusdr import graph
    desc, kind, L, T, D, cutoff, window, fs = WORKLOADS["c3"]
    taps = lowpass(T, cutoff, window)
    n_out = (L - T) // D + 1
    out = {"workload": "C3 through the filter-graph nodes: Fir(Float taps, FloatComplex, D=10) -> QuadAmDemod -> "
                       "device sink, SteppingDriver.doFilter, one 2^28-sample segment per step",
           "kernel_line_msps": kernel_value}
    steps = segments - warmup
    # full C3-sized launches before each timed node run, as the kernel line settles: the clock under
    # the board's power cap only reaches its steady state after ~10-20 ms of full load, and a
    # lighter settle would time the first steps at a burst clock the kernel line never sees
    probe_n = n_out
    taps_d = torch.from_numpy(taps).to(device)
    probe_x = torch.zeros((probe_n - 1) * D + T, dtype=torch.complex64, device=device)
    probe_out = torch.empty(probe_n, dtype=torch.float32, device=device)
    for fuse in (True, False):
        q = graph.Queue(device.index)
        fir = graph.Node.fir(q, taps, D, graph.SAMPLE_FLOAT_COMPLEX)
        am = graph.Node.quad_am_demod(q)
        sink = graph.Node.device_sink(q, n_out * 4)
        drv = graph.SteppingDriver()
        drv.set_fuse_fir_am(fuse)
        drv.connect(fir, 0, am, 0)
        drv.connect(am, 0, sink, 0)
        n_in = segments * n_out * D + T - D
        x = torch.empty(n_in, dtype=torch.complex64, device=device)
        ops.synth_wideband_cf32(0xC3, 0.013, 0.31, 0, n_in, out=x)
        torch.cuda.synchronize()
        fir.push_device(x.data_ptr(), x.numel() * 8)
        q.sync()
        del x
        for _ in range(warmup):
            drv.do_filter()
        q.sync()
        settle(lambda: ops.fir(taps_d, probe_x, D, probe_n, out=probe_out, am=True), SETTLE_S)
        # outputs through the WHOLE chain in the timed steps: the fewer of the FIR outputs computed
        # and the AM outputs computed in them. Unfused, the Fir fills the AM window ahead by its
        # headroom (2-3 segments per launch), so the AM stage alone also drains what the Fir computed
        # during warm-up; r03 counted those AM outputs and credited the timed steps with FIR work
        # done before them (583 Gs/s "unfused" > the kernel line: 3 FIR launches of ~60 M outputs
        # in 10 timed steps, rocprof trace profiles/r04/exp/nodes_trace_summary.txt)
        fir0, am0 = fir.output_size()[0] // 8, am.output_size()[0] // 4
        t0 = time.perf_counter()
        for _ in range(steps):
            drv.do_filter()
        q.sync()
        dt = (time.perf_counter() - t0) / steps
        fir_done = fir0 - fir.output_size()[0] // 8           # FIR outputs computed (Fir input consumed)
        am_done = fir_done - (am.output_size()[0] // 4 - am0)  # AM outputs computed (AM input consumed)
        done = min(fir_done, am_done)
        msps = done * D / steps / dt / 1e6
        st = drv.graph_stats()
        key = "fused" if fuse else "unfused"
        out[key] = {"value": msps, "unit": "Msamples/s", "ms_per_step": dt * 1e3,
                    "outputs_per_step": done / steps, "fir_outputs": fir_done, "am_outputs": am_done,
                    "fused_edges": st["fused"],
                    "vs_kernel_line": msps / kernel_value}
        del drv, sink, am, fir
        torch.cuda.empty_cache()
    out["host_step_1MiB"] = host_step_costs(ops, device)
    return out


def stream_path(ops, device, kernel_value, chunk=(1 << 22) - 4, steps=256, warmup=48, n_src=12):
    """C3 at SURVEY 8(d)'s streaming granularity (VERDICT r05 missing 3): a live 200 Msps receiver's chain
    through the reference's node API - Fir(real taps, FloatComplex, D = 10) -> QuadAmDemod -> device sink -
    stepped one ~2^22-sample push at a time (chunk = 2^22 - 4, a multiple of D, so the chain's state repeats
    and the steady-state steps replay cached hipGraphs: SteppingDriver.doFilterGraphed; the reference steps
    1 MiB chunks, SteppingDriver.cpp:284-287). Each step = the upstream's write of the chunk into the Fir's
    input window (push_device: a D2D copy from one of `n_src` source buffers, 32 MB each, rotated past the
    Infinity Cache) + one replayed step (the fused Fir -> AM launch). Timed: `steps` steps back to back, no
    host sync inside; value = input Msamples/s. Host microseconds per step (push + replay) from a separate
    synchronised loop."""
    from gpusdr import graph
    desc, kind, L, T, D, cutoff, window, fs = WORKLOADS["c3"]
    taps = lowpass(T, cutoff, window)
    q = graph.Queue(device.index)
    fir = graph.Node.fir(q, taps, D, graph.SAMPLE_FLOAT_COMPLEX)
    am = graph.Node.quad_am_demod(q)
    sink = graph.Node.device_sink(q, 0)
    drv = graph.SteppingDriver()
    drv.connect(fir, 0, am, 0)
    drv.connect(am, 0, sink, 0)
    srcs = []
    for k in range(n_src):
        x = torch.empty(chunk, dtype=torch.complex64, device=device)
        ops.synth_wideband_cf32(0xC3, 0.013, 0.31, k * chunk, chunk, out=x)
        srcs.append(x)
    torch.cuda.synchronize()
    i = 0

    def step():
        nonlocal i
        x = srcs[i % n_src]
        i += 1
        fir.push_device(x.data_ptr(), chunk * 8)
        drv.do_filter_graphed(q)

    for _ in range(warmup):
        step()
    q.sync()
    settle(step, SETTLE_S)
    q.sync()
    a0 = am.output_size()[0]
    ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
    ev[0].record(torch.cuda.ExternalStream(q.stream))
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    ev[1].record(torch.cuda.ExternalStream(q.stream))
    q.sync()
    dt = (time.perf_counter() - t0) / steps
    gpu_ms = ev[0].elapsed_time(ev[1]) / steps
    host = []
    for _ in range(64):
        t1 = time.perf_counter()
        step()
        host.append(time.perf_counter() - t1)
        q.sync()
    st = drv.graph_stats()
    msps = chunk / dt / 1e6
    out = {"workload": f"C3 as a live stream: Fir(Float taps, FloatComplex, D=10) -> QuadAmDemod -> device sink, "
                       f"{chunk}-sample pushes (2^22 - 4, a multiple of D), one replayed hipGraph step each "
                       "(SteppingDriver.doFilterGraphed); the push (upstream D2D write into the Fir window) included",
           "value": msps, "unit": "Msamples/s", "samples_per_step": chunk, "steps": steps,
           "ms_per_step": dt * 1e3, "gpu_ms_per_step": gpu_ms,
           "host_us_per_step": float(np.median(host[16:])) * 1e6,
           "vs_kernel_line": msps / kernel_value,
           "graph": st}
    del drv, sink, am, fir, srcs
    torch.cuda.empty_cache()
    return out


def host_step_costs(ops, device, steps=60):
    """Host time of one SteppingDriver step of the fused C3 chain (Fir -> QuadAmDemod -> device
    sink) at the reference's 1 MiB chunk: doFilter (eager) vs doFilterGraphed (replay), medians of
    the second half of `steps` pushes."""
    from gpusdr import graph
    desc, kind, L, T, D, cutoff, window, fs = WORKLOADS["c3"]
    taps = lowpass(T, cutoff, window)
    q = graph.Queue(device.index)
    chunk = 131_070  # cf32 samples, a multiple of D: the chain's state repeats
    xs = torch.empty(chunk, dtype=torch.complex64, device=device)
    ops.synth_wideband_cf32(0xC3, 0.013, 0.31, 0, chunk, out=xs)
    host = {}
    for mode in ("eager", "graphed"):
        fir = graph.Node.fir(q, taps, D, graph.SAMPLE_FLOAT_COMPLEX)
        am = graph.Node.quad_am_demod(q)
        sink = graph.Node.device_sink(q, 0)
        drv = graph.SteppingDriver()
        drv.connect(fir, 0, am, 0)
        drv.connect(am, 0, sink, 0)
        ts = []
        for i in range(steps):
            fir.push_device(xs.data_ptr(), chunk * 8)
            t0 = time.perf_counter()
            drv.do_filter() if mode == "eager" else drv.do_filter_graphed(q)
            ts.append(time.perf_counter() - t0)
            q.sync()
        host[mode] = {"host_us_per_step": float(np.median(ts[steps // 2:])) * 1e6, **drv.graph_stats()}
    return host


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default="c3", choices=sorted(WORKLOADS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--c5-mode", default="sharded", choices=["sharded", "resident", "chunked"],
                    help="c5: the time-sharded chain with its cascaded halo (default); or the gsdrAmChain "
                         "executor: one graph over the resident 1 s segment / one graph per 5 M-sample chunk "
                         "(N = 1 semantics: at N > 1 those run replicas)")
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="torch.distributed backend for the halo ring (nccl = RCCL over xGMI; gloo stages "
                         "halos through host memory)")
    ap.add_argument("--share-gpu", action="store_true",
                    help="run every rank on cuda:0 (testing the multi-rank path on a one-GPU box; gloo)")
    ap.add_argument("--no-extras", action="store_true",
                    help="skip the secondary measurements (C4 strong scaling, C5, C2, the C3 node path and stream) that the "
                         "default run adds to its JSON line under 'extras'")
    ap.add_argument("--kernel-policy", type=int, default=0,
                    help="gsdrAmdSetKernelPolicy flags for A/B runs (e.g. 64 = GSDR_POLICY_I8_WS8, the r04 8-way int8 "
                         "kernel); recorded in the line's config when nonzero")
    args = ap.parse_args()
    if args.share_gpu and args.backend != "gloo":
        raise SystemExit("bench.py: --share-gpu needs --backend gloo (RCCL runs one rank per GPU)")

    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        spawn_ranks(args.gpus, args.share_gpu)
        return
    rank, world, local = dist_setup(args.gpus, args.backend, args.share_gpu)
    device = torch.device("cuda", local)
    stage = args.backend != "nccl"
    from gpusdr import ops
    if args.kernel_policy:
        global KERNEL_POLICY
        KERNEL_POLICY = args.kernel_policy
        ops.set_kernel_policy(args.kernel_policy)
    if args.workload == "c5":
        chain = (AmChainSharded(ops, rank, world, device, stage) if args.c5_mode == "sharded" else
                 AmChainRunner(ops, rank, world, device, args.c5_mode))
    else:
        chain = ShardedChain(ops, args.workload, rank, world, device, stage)

    elapsed, kernel_ms, direct_blocks = timed_steps(chain, args.steps, args.warmup, world, args.backend, device,
                                                    local, ops)
    bytes_, (compute_kind, ops_, peak_t) = chain.timed_bytes_ops()
    achieved_gbs = bytes_ / (kernel_ms * 1e-3) / 1e9
    achieved_t = ops_ / (kernel_ms * 1e-3) / 1e12
    total_samples = world * chain.L * args.steps
    value = total_samples / elapsed / 1e6

    # secondary workloads in the same run, so the driver's 1/2/4/8-GPU runs measure every config
    # BASELINE.json names: C4 as stated (one 2^30-sample stream split over the GPUs, strong scaling),
    # the C5 chain, C2 (configs[1], the HackRF-shaped int8 chain), and (N = 1) C3 through the
    # reference's node API
    extras = {}
    if args.workload == "c3" and not args.no_extras:
        if world == 1:
            extras["c3_mixed"] = mixed_vs_plain(ops, chain)
        chain_info = (chain.kernel_class, kernel_name(chain), chain.L, chain.T, chain.D, chain.kind, chain.geom,
                      getattr(chain, "n_slots", 1))
        del chain
        torch.cuda.empty_cache()
        for wl, k, w in (("c4s", 6, 2), ("c5", 40, 3), ("c2", 400, 5)):
            xc = (AmChainSharded(ops, rank, world, device, stage) if wl == "c5" else
                  ShardedChain(ops, wl, rank, world, device, stage))
            e2, k2, _ = timed_steps(xc, k, w, world, args.backend, device, local, ops)
            extras[wl] = extra_line(wl, xc, e2, k2, k, world)
            del xc
            torch.cuda.empty_cache()
        if world == 1:
            extras["c3_nodes"] = node_path(ops, device, value)
            extras["c3_stream"] = stream_path(ops, device, value)
            extras["c5_host_fed"] = host_fed_c5(device)
        chain = argparse.Namespace(kernel_class=chain_info[0], L=chain_info[2], T=chain_info[3], D=chain_info[4],
                                   kind=chain_info[5], geom=chain_info[6], n_slots=chain_info[7])
        kernel_label = chain_info[1]
    else:
        kernel_label = kernel_name(chain)
    # measured bandwidth in this process, the second reference of the roofline
    probe = hbm_probe(ops, device) if not args.no_extras else None

    if rank == 0:
        desc = WORKLOADS[args.workload][0]
        cpu = None
        if world == 1 and not args.no_cpu_baseline:
            cpu = cpu_baseline(args.workload)
        traffic, traffic_src = load_traffic(args.workload)
        rf_traffic = None
        if args.workload == "c5" and not (world == 1 and args.c5_mode == "sharded"):
            # the PMC summary is of the fused N = 1 step's one launch; elsewhere the timed region
            # holds more launches (bulk + head, or an executor graph): kept apart, labelled by source
            rf_traffic, traffic = traffic, None
        if world > 1 and traffic is not None:
            # profiled at N = 1 (one launch over the whole step); at N > 1 the timed launch is the bulk
            # part, a different size: the per-launch figure is that configuration's, labelled
            rf_traffic, traffic = traffic, None
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "strong" if args.workload in STRONG else "weak",
            "vs_baseline": None,
            "dtype": "f32",  # complex float32 samples / fp32 accumulation; the arithmetic form:
            "arithmetic": compute_kind,
            "data": "synthetic (deterministic splitmix64 + tone generator, generated in HBM)",
            "config": {
                "workload": desc,
                "samples_per_gpu_step": chain.L,
                "taps": chain.T,
                "decimation": chain.D,
                "input": "int8 IQ" if chain.kind == "i8" else "cf32",
                "parallelism": ("disjoint time ranges per rank, history primed by warm-up (no collective)"
                                if chain.geom is None else
                                f"time-shard x{world} (ring halo of {chain.geom.halo} samples over "
                                f"{'RCCL' if args.backend == 'nccl' else args.backend + ', host-staged'}"
                                f"{', ranks sharing cuda:0' if args.share_gpu else ''})")
                if world > 1 else f"single GPU (halo = own history carry, {chain.geom.halo if chain.geom else 0} samples)",
                "buffer_sets": getattr(chain, "n_slots", 1),
                **({"kernel_policy": args.kernel_policy} if args.kernel_policy else {}),
                **({"c5_mode": chain.mode, "audio_taps": chain.Ta, "audio_decimation": chain.Da}
                   if args.workload == "c5" else {}),
            },
            "roofline": {
                "bound": "hbm",
                "kernel": kernel_label,
                "achieved": achieved_gbs,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved_gbs / HBM_PEAK_GBS,
                "traffic": traffic,
                **({"traffic_of_profiled_config": rf_traffic} if rf_traffic is not None else {}),
                "traffic_source": traffic_src,
                **({"measured_read_gbs": probe["read_gbs"], "measured_copy_gbs": probe["copy_gbs"],
                    "frac_of_measured_read": achieved_gbs / probe["read_gbs"],
                    "frac_of_measured_copy": achieved_gbs / probe["copy_gbs"]} if probe else {}),
                "avg_launch_ms": kernel_ms,
                "algorithmic_bytes_per_launch": bytes_,
                "compute": {"kind": compute_kind, "achieved_tflops": achieved_t, "peak_tflops": peak_t,
                            "frac": achieved_t / peak_t, "flops_per_launch": ops_},
                "kernel_class": chain.kernel_class,
                "fft_direct_blocks": direct_blocks,
            },
            "cpu_baseline": cpu,
            **({"extras": extras} if extras else {}),
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
