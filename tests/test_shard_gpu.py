"""Time-sharded streams on the HIP kernels: 2, 4 and 8 ranks (gloo, halos staged through host
memory), all on cuda:0, run the ring-halo protocol of gpusdr/shard.py with the real gfx950 FIR
kernels - C4's shape (cf32, 1023 taps, D = 1, bulk / head launches) at the config's 2 and 4 ranks,
and the C5 AM receive chain with its cascaded halo ((Ta - 1) D + T - 1 samples, AmChainShard) at 2
and the config's 8 ranks. The concatenated per-rank outputs must
equal the float64 oracle over the whole stream within the FIR tolerance 1e-6 * sum|h||x|
(SURVEY.md 8d), i.e. sharding changes nothing but where work runs. The stream is primed: rank 0's
first halo holds the stream's first samples (as a live receiver's history would), so no window
is artificially zero-padded.
The same code runs over RCCL with one GPU per rank in bench.py.
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIR_TOL = 1e-6
STEPS = 3


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, kind, out_dir):
    import sys
    sys.path[:0] = [os.path.join(REPO, "cuda-sdr_amd"), os.path.join(REPO, "oracle")]
    import torch
    import torch.distributed as dist

    import oracle as orc
    from gpusdr import ops
    from gpusdr.shard import AmChainShard, ChainShardGeometry, HaloRing, ShardGeometry

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    # up to 8 processes time-share one GPU here, so a wave-specialised kernel's hand-off wait can be
    # stalled far longer than on a GPU of its own: give them room, and fail loudly on any abort
    ops.set_ws_spin_limit(1 << 28)
    ops.ws_aborts(reset=True)
    if os.environ.get("GSDR_TEST_POLICY"):  # diagnostics: run the ranks under a kernel policy
        ops.set_kernel_policy(int(os.environ["GSDR_TEST_POLICY"]))
    outs = []
    if kind == "c4":
        T, D, L = 1023, 1, 20_000
        geom = ShardGeometry(rank, world, L, T, D)
        taps = torch.from_numpy(orc.lowpass_taps(T, 0.04, "blackman")).to(dev)
        H = geom.halo
        buf = torch.zeros(H + L, dtype=torch.complex64, device=dev)
        seg = buf[H:]
        incoming = torch.zeros(H, dtype=torch.complex64, device=dev) if rank == 0 else None
        ring = HaloRing(geom, buf[:H], seg[L - H:], incoming, stage=True)
        y = torch.empty(geom.outputs, dtype=torch.complex64, device=dev)
        hb = geom.head_outputs
        primed = None
        if rank == 0:
            ops.synth_wideband_cf32(0xC4, 0.013, 0.31, 0, H, out=buf[:H])  # primed history
            primed = buf[:H].cpu().numpy().copy()
        inputs = []
        for step in range(STEPS):
            ops.synth_wideband_cf32(0xC4, 0.013, 0.31, H + geom.segment_start(step), L, out=seg)
            inputs.append(seg.cpu().numpy().copy())
            ring.step(lambda: ops.fir(taps, seg[geom.bulk_input_offset():], D, geom.outputs - hb, out=y[hb:]),
                      lambda: ops.fir(taps, buf, D, hb, out=y[:hb]))
            torch.cuda.synchronize()
            outs.append(y.cpu().numpy().copy())
    else:
        T, D, Ta, Da, L = 1023, 10, 255, 20, 40_000
        geom = ChainShardGeometry(rank, world, L, T, D, Ta, Da)
        rf = torch.from_numpy(orc.lowpass_taps(T, 0.04, "blackman")).to(dev)
        au = torch.from_numpy(orc.lowpass_taps(Ta, 0.02)).to(dev)
        sh = AmChainShard(geom, rf, au, dev, stage=True)
        H = geom.halo
        primed = None
        if rank == 0:
            ops.synth_iq_int8(0x5EED, 1e9, 1e3, 7.5e7, 0, H, out=sh.buf[: 2 * H])  # primed history
            primed = sh.buf[: 2 * H].cpu().numpy().copy()
        inputs = []
        for step in range(STEPS):
            ops.synth_iq_int8(0x5EED, 1e9, 1e3, 7.5e7, H + geom.segment_start(step), L, out=sh.seg)
            inputs.append(sh.seg.cpu().numpy().copy())
            out = sh.step()
            torch.cuda.synchronize()
            outs.append(out.cpu().numpy().copy())
    aborts = ops.ws_aborts(reset=True)
    if aborts:
        raise RuntimeError(f"rank {rank}: {aborts} wave-specialised hand-off aborts")
    np.save(os.path.join(out_dir, f"{kind}_rank{rank}.npy"), np.stack(outs))
    # the stream as the GPU generated it (the oracle's float64 chain runs on exactly these samples:
    # the host restatement of the synthetic source may round a rare int8 sample to the neighbouring
    # code - GPU sincos vs libm in the last ulp - which is not what this test is about)
    np.save(os.path.join(out_dir, f"{kind}_in_rank{rank}.npy"), np.stack(inputs))
    if rank == 0:
        np.save(os.path.join(out_dir, f"{kind}_halo.npy"), primed)
    dist.barrier()
    dist.destroy_process_group()


def _run(kind, tmp_path, world):
    """(outputs in stream order, the input stream the ranks generated: primed halo + segments)."""
    import torch.multiprocessing as mp
    mp.start_processes(_rank_main, args=(world, _free_port(), kind, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    per = [np.load(os.path.join(tmp_path, f"{kind}_rank{r}.npy")) for r in range(world)]
    ins = [np.load(os.path.join(tmp_path, f"{kind}_in_rank{r}.npy")) for r in range(world)]
    stream = np.concatenate([np.load(os.path.join(tmp_path, f"{kind}_halo.npy"))] +
                            [ins[r][s] for s in range(STEPS) for r in range(world)])
    return np.concatenate([per[r][s] for s in range(STEPS) for r in range(world)]), stream


@pytest.mark.parametrize("world", [2, 4])
def test_c4_shape_time_sharded_on_hip(tmp_path, orc, world):
    T, D, L = 1023, 1, 20_000
    got, stream = _run("c4", tmp_path, world)
    n = L * world * STEPS
    assert len(stream) == T - 1 + n
    y64, bound = orc.fir_f64(orc.lowpass_taps(T, 0.04, "blackman"), stream, D, n // D)
    assert len(got) == len(y64)
    err = np.abs(got.astype(np.complex128) - y64)
    assert np.all(err <= FIR_TOL * bound + 1e-30), float(np.max(err / (bound + 1e-30)))


@pytest.mark.parametrize("world", [1, 2, 8])  # 1: the single-rank step is ONE fused launch
def test_c5_chain_time_sharded_cascaded_halo(tmp_path, orc, world):
    from gpusdr.shard import ChainShardGeometry
    T, D, Ta, Da, L = 1023, 10, 255, 20, 40_000
    H = ChainShardGeometry(0, world, L, T, D, Ta, Da).halo
    assert H == 3600  # (Ta - 1) D + T - 1 = 3562, rounded up to a multiple of D Da
    got, padded = _run("c5", tmp_path, world)  # the primed stream the ranks generated
    assert len(padded) == 2 * (H + L * world * STEPS)
    rf, au = orc.lowpass_taps(T, 0.04, "blackman"), orc.lowpass_taps(Ta, 0.02)
    x = orc.int8_to_float(padded).view(np.complex64)
    y, rf_bound = orc.fir_f64(rf, x, D)
    am = np.abs(y)
    want, audio_bound = orc.fir_f64(au, am.astype(np.float32), Da)
    n = len(got)
    assert n == L * world * STEPS // (D * Da) and len(want) >= n
    carried, _ = orc.fir_f64(np.abs(au), (FIR_TOL * (rf_bound + am)).astype(np.float32), Da, n)
    bound = carried + FIR_TOL * audio_bound[:n] + 1e-30
    bad = np.nonzero(np.abs(got - want[:n]) > bound)[0]
    per = L // (D * Da)  # outputs per rank per step
    assert len(bad) == 0, (len(bad), [(int(i), int(i // per % world), int(i // per // world), float(got[i]),
                                       float(want[i]), float(bound[i])) for i in bad[:6]])


def test_c5_chain_single_rank_one_launch_matches_split(orc):
    """World 1: AmChainShard runs the RF stage as one launch over [halo | segment]. Against the bulk +
    head split the outputs may differ in the last bits (the matrix-core kernel's tiles start 360
    outputs apart, so an output's split-K partial sums group its taps differently); both meet the
    float64 chain within the carried tolerance."""
    import torch
    from gpusdr import ops
    from gpusdr.shard import AmChainShard, ChainShardGeometry
    T, D, Ta, Da, L = 1023, 10, 255, 20, 40_000
    dev = torch.device("cuda", 0)
    geom = ChainShardGeometry(0, 1, L, T, D, Ta, Da)
    rf = torch.from_numpy(orc.lowpass_taps(T, 0.04, "blackman")).to(dev)
    au = torch.from_numpy(orc.lowpass_taps(Ta, 0.02)).to(dev)
    H = geom.halo
    one = AmChainShard(geom, rf, au, dev)
    split = AmChainShard(geom, rf, au, dev)
    for sh in (one, split):
        ops.synth_iq_int8(0x5EED, 1e9, 1e3, 7.5e7, 0, H, out=sh.buf[: 2 * H])
    got, ref = [], []
    for step in range(3):
        for sh in (one, split):
            ops.synth_iq_int8(0x5EED, 1e9, 1e3, 7.5e7, H + geom.segment_start(step), L, out=sh.seg)
        got.append(one.step().cpu().numpy().copy())
        split.ring.step(split._bulk, split._head)
        ops.fir(au, split.am, Da, geom.outputs, out=split.out)
        ref.append(split.out.cpu().numpy().copy())
    got, ref = np.concatenate(got), np.concatenate(ref)
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-7)
    padded = orc.synth_iq_int8(0x5EED, 1e9, 1e3, 7.5e7, 0, H + 3 * L)
    x = orc.int8_to_float(padded).view(np.complex64)
    y, rf_bound = orc.fir_f64(orc.lowpass_taps(T, 0.04, "blackman"), x, D)
    am = np.abs(y)
    want, audio_bound = orc.fir_f64(orc.lowpass_taps(Ta, 0.02), am.astype(np.float32), Da)
    n = len(got)
    carried, _ = orc.fir_f64(np.abs(orc.lowpass_taps(Ta, 0.02)), (FIR_TOL * (rf_bound + am)).astype(np.float32), Da, n)
    for out in (got, ref):
        assert np.all(np.abs(out - want[:n]) <= carried + FIR_TOL * audio_bound[:n] + 1e-30)


def test_c5_ring_views_read_history_in_place(orc):
    """World 1 with the slots as consecutive views of one input ring (bench.py's C5 layout): slot
    k + 1's halo IS slot k's segment tail, so step(carry=False) copies nothing, and the audio equals
    one chain stepping its own buffer with the history copy, bit for bit."""
    import torch
    from gpusdr import ops
    from gpusdr.shard import AmChainShard, ChainShardGeometry
    T, D, Ta, Da, L = 1023, 10, 255, 20, 40_000
    dev = torch.device("cuda", 0)
    geom = ChainShardGeometry(0, 1, L, T, D, Ta, Da)
    H = geom.halo
    rf = torch.from_numpy(orc.lowpass_taps(T, 0.04, "blackman")).to(dev)
    au = torch.from_numpy(orc.lowpass_taps(Ta, 0.02)).to(dev)
    ring = torch.zeros(2 * (H + 3 * L), dtype=torch.int8, device=dev)
    views = [AmChainShard(geom, rf, au, dev, buf=ring[2 * k * L: 2 * (k * L + H + L)]) for k in range(3)]
    ops.synth_iq_int8(0x5EED, 1e9, 1e3, 7.5e7, 0, H + 3 * L, out=ring)  # history + three segments in place
    one = AmChainShard(geom, rf, au, dev)
    one.buf[: 2 * H].copy_(ring[: 2 * H])
    got, ref = [], []
    for k in range(3):
        got.append(views[k].step(carry=False).cpu().numpy().copy())
        one.seg.copy_(views[k].seg)
        ref.append(one.step().cpu().numpy().copy())
    assert np.array_equal(np.concatenate(got), np.concatenate(ref))
