"""The native time-sharded stream executor (gsdrShardStream*, gpusdr/native_shard.py): the halo-ring
step of gpusdr/shard.py in C++, its exchange supplied by the caller. 1, 2 and 4 ranks (gloo ranks on
cuda:0, the halo staged through host memory by a Python exchange hook) with the real gfx950 FIR
kernels - cf32 on the FFT kernel (C4's 1023 taps, D = 1; C3's D = 10) and int8 IQ with AM on the
matrix-core kernel - must reproduce the float64 oracle over the whole primed stream within the FIR
tolerance 1e-6 * sum|h||x|, the same bar as tests/test_shard_gpu.py."""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIR_TOL = 1e-6
STEPS = 3
CASES = {  # name: (int8 IQ, AM, taps, D, segment samples)
    "c4": (False, False, 1023, 1, 20_000),
    "c3": (False, True, 1023, 10, 30_000),
    "i8": (True, True, 255, 4, 16_000),
}


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _stream_piece(ops, torch, i8, start, n, dev):
    """Samples [start, start + n) of the test stream, generated on the GPU."""
    if i8:
        x = torch.empty(2 * n, dtype=torch.int8, device=dev)
        ops.synth_iq_int8(0x5EED, 1e9, 1e3, 7.5e7, start, n, out=x)
    else:
        x = torch.empty(n, dtype=torch.complex64, device=dev)
        ops.synth_wideband_cf32(0xC4, 0.013, 0.31, start, n, out=x)
    return x


def _rank_main(rank, world, port, case, out_dir, transport="host"):
    import sys
    sys.path[:0] = [os.path.join(REPO, "cuda-sdr_amd"), os.path.join(REPO, "oracle")]
    import torch
    import torch.distributed as dist

    import oracle as orc
    from gpusdr import ops
    from gpusdr.native_shard import RcclComm, ShardStream, host_staged_exchange

    i8, am, T, D, L = CASES[case]
    if world > 1:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", 0)
    ops.set_ws_spin_limit(1 << 28)  # several ranks time-share the GPU
    ops.ws_aborts(reset=True)
    taps = orc.lowpass_taps(T, 0.04, "blackman")
    comm = None
    if transport == "rccl":  # one communicator of `world` ranks (world 1: a ring of one, self send / recv)
        torch.cuda.set_device(dev)
        if world > 1:
            raise NotImplementedError("RCCL needs one GPU per rank; this box has one")
        comm = RcclComm(world, RcclComm.unique_id(), rank, 0)
        # the raw hook first: a byte halo sent to this rank itself arrives intact
        n = 8190
        send = torch.randint(0, 256, (n,), dtype=torch.uint8, device=dev)
        recv = torch.zeros(n, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize()
        comm.exchange(send.data_ptr(), recv.data_ptr(), n, rank, rank, torch.cuda.current_stream(dev).cuda_stream)
        torch.cuda.synchronize()
        if not torch.equal(send, recv):
            raise RuntimeError("RCCL self exchange: received bytes differ from the sent ones")
        exchange = comm
    else:
        exchange = host_staged_exchange() if world > 1 else None
    sh = ShardStream(rank, world, taps, D, L, int8_iq=i8, am=am, exchange=exchange)
    H = T - 1
    if rank == 0:  # the stream's first H samples are the primed history of rank 0's first step
        sh.write_halo(_stream_piece(ops, torch, i8, 0, H, dev))
    outs = []
    for step in range(STEPS):
        start = H + (step * world + rank) * L
        sh.write_segment(_stream_piece(ops, torch, i8, start, L, dev))
        y = sh.step()
        torch.cuda.synchronize()
        outs.append(y.cpu().numpy().copy())
    aborts = ops.ws_aborts(reset=True)
    if aborts:
        raise RuntimeError(f"rank {rank}: {aborts} wave-specialised hand-off aborts")
    if comm is not None:  # the communicator cannot be destroyed under a live executor
        try:
            comm.close()
        except RuntimeError:
            pass
        else:
            raise RuntimeError("RcclComm.close succeeded while a ShardStream still used it")
    sh.close()
    if comm is not None:
        comm.close()
        if comm.handle:
            raise RuntimeError("RcclComm.close left the handle set")
    np.save(os.path.join(out_dir, f"{case}_rank{rank}.npy"), np.stack(outs))
    if rank == 0:  # the whole stream as the GPU generates it, for the oracle
        full = _stream_piece(ops, torch, i8, 0, H + world * STEPS * L, dev)
        np.save(os.path.join(out_dir, f"{case}_stream.npy"), full.cpu().numpy())
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def _check_against_oracle(orc, tmp_path, case, world):
    i8, am, T, D, L = CASES[case]
    per = [np.load(os.path.join(tmp_path, f"{case}_rank{r}.npy")) for r in range(world)]
    got = np.concatenate([per[r][s] for s in range(STEPS) for r in range(world)])
    stream = np.load(os.path.join(tmp_path, f"{case}_stream.npy"))
    x = orc.int8_to_float(stream).view(np.complex64) if i8 else stream
    n = world * STEPS * L // D
    assert len(got) == n
    y64, bound = orc.fir_f64(orc.lowpass_taps(T, 0.04, "blackman"), x, D, n)
    want = np.abs(y64) if am else y64
    err = np.abs(got.astype(np.complex128) - want)
    assert np.all(err <= FIR_TOL * bound + 1e-30), float(np.max(err / (bound + 1e-30)))


@pytest.mark.parametrize("case,world", [("c4", 1), ("c4", 2), ("c4", 4), ("c3", 2), ("i8", 1), ("i8", 2)])
def test_native_shard_stream_matches_oracle(tmp_path, orc, case, world):
    import torch.multiprocessing as mp
    mp.start_processes(_rank_main, args=(world, _free_port(), case, str(tmp_path)), nprocs=world, join=True,
                       start_method="spawn")
    _check_against_oracle(orc, tmp_path, case, world)


@pytest.mark.parametrize("case", ["c4", "i8"])
def test_native_shard_stream_rccl_ring_of_one(tmp_path, orc, case):
    """the RCCL path executed on the one GPU the box has. In a fresh process the
    library makes a 1-rank communicator (gsdrShardRcclGetUniqueId / CommCreate), sends a byte halo to
    itself through gsdrShardExchangeRccl (grouped ncclSend / ncclRecv on a stream) and gets it back
    intact; then a world-1 ShardStream whose hook IS gsdrShardExchangeRccl runs the ring protocol on a
    ring of one (bulk launch beside the RCCL transfer on the exchange stream, head from the halo
    received a step earlier) and must match the float64 oracle. Multi-GPU RCCL stays unmeasured until
    the driver's 8-GPU node runs it."""
    import torch.multiprocessing as mp
    mp.start_processes(_rank_main, args=(1, _free_port(), case, str(tmp_path), "rccl"), nprocs=1, join=True,
                       start_method="spawn")
    _check_against_oracle(orc, tmp_path, case, 1)


def test_native_shard_async_exchange_two_ranks_one_process(orc):
    """an exchange that only ENQUEUES its transfers and returns. Two ranks of a
    2-rank ring live in one process on cuda:0; rank 0's hook puts a ~1 ms spin kernel on its exchange
    stream, then the two halo copies (its tail -> rank 1's halo, rank 1's tail -> its incoming buffer)
    and records an event; rank 1's hook makes its exchange stream wait for that event. So the bulk
    launches run while the halo writes are still pending, rank 1's head must wait on its 'exchanged'
    event and rank 0 must copy its incoming halo only after the transfer: an ordering bug in the
    segReady / exchanged events or the rank-0 incoming -> halo copy reads a stale halo and fails the
    float64 comparison."""
    import ctypes

    import torch

    from gpusdr import ops
    from gpusdr.native_shard import ShardStream, _L

    case, world = "c3", 2
    i8, am, T, D, L = CASES[case]
    dev = torch.device("cuda", 0)
    taps = orc.lowpass_taps(T, 0.04, "blackman")
    H = T - 1
    ranks = {}
    done = torch.cuda.Event()
    lib = _L()

    def hook0(send_tail, recv_halo, nbytes, next_rank, prev_rank, xstream):
        xs = torch.cuda.ExternalStream(xstream, device=dev)
        with torch.cuda.stream(xs):
            torch.cuda._sleep(2_000_000)  # the transfer stays pending while the bulk launches run
        for dst, src in ((ranks[1].halo_ptr, send_tail), (recv_halo, ranks[1].tail_ptr)):
            code = lib.hipMemcpyAsync(ctypes.c_void_p(dst), ctypes.c_void_p(src), nbytes, 3, ctypes.c_void_p(xstream))
            if code != 0:
                raise RuntimeError(f"hipMemcpyAsync {code}")
        done.record(xs)

    def hook1(send_tail, recv_halo, nbytes, next_rank, prev_rank, xstream):
        torch.cuda.ExternalStream(xstream, device=dev).wait_event(done)

    ranks[0] = ShardStream(0, world, taps, D, L, int8_iq=i8, am=am, exchange=hook0)
    ranks[1] = ShardStream(1, world, taps, D, L, int8_iq=i8, am=am, exchange=hook1)
    ranks[0].write_halo(_stream_piece(ops, torch, i8, 0, H, dev))
    outs = {0: [], 1: []}
    for step in range(STEPS):
        for r in (0, 1):
            ranks[r].write_segment(_stream_piece(ops, torch, i8, H + (step * world + r) * L, L, dev))
        ys = [ranks[r].step() for r in (0, 1)]
        torch.cuda.synchronize()
        for r in (0, 1):
            outs[r].append(ys[r].cpu().numpy().copy())
    for r in (0, 1):
        ranks[r].close()
    got = np.concatenate([outs[r][s] for s in range(STEPS) for r in range(world)])
    x = _stream_piece(ops, torch, i8, 0, H + world * STEPS * L, dev).cpu().numpy()
    n = world * STEPS * L // D
    y64, bound = orc.fir_f64(taps, x, D, n)
    err = np.abs(got.astype(np.complex128) - (np.abs(y64) if am else y64))
    assert np.all(err <= FIR_TOL * bound + 1e-30), float(np.max(err / (bound + 1e-30)))


def test_native_shard_stream_rejects_bad_shapes():
    from gpusdr.native_shard import ShardStream
    with pytest.raises(RuntimeError):
        ShardStream(0, 1, np.ones(8, np.float32), 3, 1000)  # L not a multiple of D
    with pytest.raises(RuntimeError):
        ShardStream(0, 2, np.ones(8, np.float32), 1, 1000)  # two ranks need an exchange


def test_native_shard_stream_failed_exchange_then_destroy(orc):
    """the failure paths of the executor. A world-1 stream whose exchange hook fails on its
    second step: that step reports the error (the bulk launch already enqueued, no head), destroy() then
    returns with nothing of the executor left pending (it waits on the events of the steps that did run),
    the device is healthy, and a fresh executor over the same stream positions matches the float64 oracle."""
    import torch

    from gpusdr import ops
    from gpusdr._native import HipError
    from gpusdr.native_shard import ShardStream

    i8, am, T, D, L = CASES["c3"]
    dev = torch.device("cuda", 0)
    taps = orc.lowpass_taps(T, 0.04, "blackman")
    H = T - 1
    calls = []

    def flaky(send_tail, recv_halo, nbytes, next_rank, prev_rank, xstream):
        calls.append(1)
        if len(calls) == 2:
            raise RuntimeError("injected exchange failure")

    s = ShardStream(0, 1, taps, D, L, int8_iq=i8, am=am, exchange=flaky)
    s.write_halo(_stream_piece(ops, torch, i8, 0, H, dev))
    s.write_segment(_stream_piece(ops, torch, i8, H, L, dev))
    s.step()
    s.write_segment(_stream_piece(ops, torch, i8, H + L, L, dev))
    with pytest.raises(HipError):
        s.step()
    s.close()
    torch.cuda.synchronize()  # nothing of the executor failed the device
    # a fresh executor: the stream from its start, checked against float64
    s = ShardStream(0, 1, taps, D, L, int8_iq=i8, am=am)  # world 1 without a hook: the history carry
    s.write_halo(_stream_piece(ops, torch, i8, 0, H, dev))
    outs = []
    for step in range(2):
        s.write_segment(_stream_piece(ops, torch, i8, H + step * L, L, dev))
        outs.append(s.step().cpu().numpy().copy())
    s.close()
    got = np.concatenate(outs)
    x = _stream_piece(ops, torch, i8, 0, H + 2 * L, dev).cpu().numpy()
    y64, bound = orc.fir_f64(taps, x, D, 2 * L // D)
    err = np.abs(got.astype(np.complex128) - np.abs(y64))
    assert np.all(err <= FIR_TOL * bound + 1e-30), float(np.max(err / (bound + 1e-30)))
