"""Time-sharded streaming (gpusdr/shard.py) with world_size 2, 4 and 8 over gloo on the CPU.

Each rank runs the real ring-halo protocol (HaloRing.step) over torch.distributed; the FIR
itself is the oracle here (the GPU path runs the same protocol with the HIP kernels in
bench.py). The halos are sent unstaged (HaloRing(stage=False)): the branch RCCL takes with device
tensors, here with host tensors (gloo cannot move device tensors; the GPU tests stage instead). The concatenated per-rank outputs must equal, bit for bit, one unsharded FIR over
the whole stream fed (T-1) zeros first - i.e. sharding changes nothing but where work runs.
"""
import os
import socket

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
L, T, STEPS = 600, 31, 4


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _segment(step, rank, world, orc):
    first = (step * world + rank) * L
    return orc.synth_wideband_cf32(0xC4, 0.013, 0.31, first, L)


def _run_rank(rank, world, port, D, out_dir):
    import sys
    sys.path[:0] = [os.path.join(REPO, "cuda-sdr_amd"), os.path.join(REPO, "oracle")]
    import torch
    import torch.distributed as dist

    import oracle as orc
    from gpusdr.shard import HaloRing, ShardGeometry

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    geom = ShardGeometry(rank, world, L, T, D)
    taps = orc.lowpass_taps(T, 0.1)
    H = geom.halo
    buf = torch.zeros(2 * (H + L), dtype=torch.float32)  # interleaved re/im: gloo moves float32
    halo, seg = buf[: 2 * H], buf[2 * H:]
    tail = seg[2 * (L - H):]
    incoming = torch.zeros(2 * H, dtype=torch.float32) if rank == 0 else None
    ring = HaloRing(geom, halo, tail, incoming)
    outs = []
    for step in range(STEPS):
        seg.copy_(torch.from_numpy(_segment(step, rank, world, orc).view(np.float32)))
        y = np.zeros(geom.outputs, dtype=np.complex128)

        def bulk():
            x = buf.numpy().view(np.complex64)[H + geom.bulk_input_offset():]
            n = geom.outputs - geom.head_outputs
            y[geom.head_outputs:], _ = orc.fir_f64(taps, x, D, n)

        def head():
            x = buf.numpy().view(np.complex64)
            y[: geom.head_outputs], _ = orc.fir_f64(taps, x, D, geom.head_outputs)

        ring.step(bulk, head)
        outs.append(y)
    np.save(os.path.join(out_dir, f"rank{rank}.npy"), np.stack(outs))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,D", [(2, 1), (2, 3), (4, 1), (8, 3)])
def test_ring_halo_matches_unsharded(tmp_path, orc, world, D):
    import torch.multiprocessing as mp
    mp.spawn(_run_rank, args=(world, _free_port(), D, str(tmp_path)), nprocs=world, join=True)
    per_rank = [np.load(os.path.join(tmp_path, f"rank{r}.npy")) for r in range(world)]
    sharded = np.concatenate([per_rank[r][s] for s in range(STEPS) for r in range(world)])
    stream = np.concatenate([_segment(s, r, world, orc) for s in range(STEPS) for r in range(world)])
    padded = np.concatenate([np.zeros(T - 1, np.complex64), stream])
    taps = orc.lowpass_taps(T, 0.1)
    ref, _ = orc.fir_f64(taps, padded, D, len(stream) // D)
    assert len(sharded) == len(ref)
    assert np.array_equal(sharded, ref)


def test_single_rank_history_carry(orc):
    """G = 1: the halo is the previous step's tail (the reference's input-window carry)."""
    import torch

    from gpusdr.shard import HaloRing, ShardGeometry
    D = 2
    geom = ShardGeometry(0, 1, L, T, D)
    H = geom.halo
    buf = torch.zeros(H + L, dtype=torch.complex64)
    ring = HaloRing(geom, buf[:H], buf[H:][L - H:])
    taps = orc.lowpass_taps(T, 0.1)
    got = []
    for step in range(3):
        buf[H:] = torch.from_numpy(_segment(step, 0, 1, orc))
        y = np.zeros(geom.outputs, np.complex128)

        def bulk():
            y[geom.head_outputs:], _ = orc.fir_f64(taps, buf.numpy()[H + geom.bulk_input_offset():], D,
                                                   geom.outputs - geom.head_outputs)

        def head():
            y[: geom.head_outputs], _ = orc.fir_f64(taps, buf.numpy(), D, geom.head_outputs)

        ring.step(bulk, head)
        got.append(y)
    stream = np.concatenate([_segment(s, 0, 1, orc) for s in range(3)])
    ref, _ = orc.fir_f64(taps, np.concatenate([np.zeros(T - 1, np.complex64), stream]), D, len(stream) // D)
    assert np.array_equal(np.concatenate(got), ref)


def test_geometry_rules():
    from gpusdr.shard import ShardGeometry
    g = ShardGeometry(1, 4, 2000, 1023, 10)
    assert g.halo == 1022 and g.outputs == 200
    assert g.head_outputs == 103 and g.bulk_input_offset() == 8  # ceil(1022/10); 103*10 - 1022
    g = ShardGeometry(2, 4, 20000, 127, 1)
    assert g.head_outputs == 126 and g.bulk_input_offset() == 0
    assert g.segment_start(3) == (3 * 4 + 2) * 20000
    assert g.next_rank == 3 and g.prev_rank == 1
    with pytest.raises(ValueError):
        ShardGeometry(0, 2, 1001, 31, 10)


def test_halo_byte_views():
    """The ring hands halos to torch.distributed as uint8 views of the same storage:
    ProcessGroupNCCL's send/recv have no complex datatype ("Unconvertible NCCL type")."""
    import torch
    from gpusdr.shard import _bytes
    x = torch.arange(12, dtype=torch.float32).to(torch.complex64)
    b = _bytes(x[3:7])
    assert b.dtype == torch.uint8 and b.numel() == 4 * 8
    b.zero_()  # same storage
    assert torch.all(x[3:7] == 0) and x[2] == 2 and x[7] == 7
    i8 = torch.arange(20, dtype=torch.int8)
    assert _bytes(i8[4:]).numel() == 16
    with pytest.raises(ValueError):
        _bytes(torch.zeros(4, 4, dtype=torch.complex64)[:, 1])


def _settle_rank(rank, world, port, out_dir):
    import sys
    import time
    sys.path[:0] = [REPO, os.path.join(REPO, "cuda-sdr_amd")]
    import torch
    import torch.distributed as dist
    torch.cuda.synchronize = lambda *a, **k: None  # CPU run: the bench's stream syncs are no-ops here
    import bench

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    count = [0]
    buf = torch.zeros(4)

    def step():  # a ring exchange per step, like the sharded chains; ranks run at different speeds
        time.sleep(0.002 * (1 + rank))
        nxt, prv = (rank + 1) % world, (rank - 1) % world
        reqs = [dist.isend(buf.clone(), nxt), dist.irecv(torch.empty(4), prv)]
        for r in reqs:
            r.wait()
        count[0] += 1

    bench.settle(step, seconds=0.08, world=world, backend="gloo")
    np.save(os.path.join(out_dir, f"settle{rank}.npy"), np.array([count[0]]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_bench_settle_same_step_count_on_every_rank(tmp_path, world):
    """bench.settle at N > 1 runs the same number of steps on every rank (each step exchanges halos;
    a rank one step short would leave its neighbour waiting for a halo - a 2-rank C5 bench hung that
    way in r04 when the settle was timed per rank)."""
    import torch.multiprocessing as mp
    mp.spawn(_settle_rank, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    counts = [int(np.load(os.path.join(tmp_path, f"settle{r}.npy"))[0]) for r in range(world)]
    assert len(set(counts)) == 1 and counts[0] >= 8, counts
