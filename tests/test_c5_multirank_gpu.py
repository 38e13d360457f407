"""The multi-rank C5 step's launches on the default (4-way) int8 kernel at the bench's size (r06).

r05 found `hipErrorIllegalAddress` in the 2- and 8-rank C5 bench (ranks sharing one MI355X) on the 4-way
kernel and routed multi-rank steps to the r04 8-way kernel. The cause: the producer waves'
window loads are inline asm the compiler does not track; after the producer loop the last loads (tiles past
the block's range) were still landing while the compiler had already handed their registers to the tail's
code - the audio output store's address among them - so a late load (late under contention: ranks sharing
the GPU) zeroed a live address. Both windows are now drained before the tail (ws_common.h
wsI8DrainWindows) and tools/isa_vmcnt_check.py proves no register is touched under a landing load
(tests/test_isa_hazards.py). These tests run exactly the launches of AmChainShard's multi-rank step
(`_bulk`: the fused chain over the segment alone, AM stored at am[360:], audio at out[18:], no AM history,
~95 tiles per block; `_head`: a one-tile, 360-output plain launch, then the head's 18 audio outputs) at the
bench's L = 125 M, against float64; once with every hand-off wait forced to give up (the abort path at this
shape); and beside concurrent HBM traffic on another stream (the co-running work that exposed the fault, and
that tripped r05's iteration-count spin limit). Reference chain: am_test.cpp:352-433, QuadAmDemod.cpp:93-98,
Fir.cpp:229-279."""
import numpy as np
import pytest

from test_am_fused import TILE, _check_audio_sampled, _sample_audio

pytestmark = pytest.mark.gpu

T, D, TA, DA, L = 1023, 10, 255, 20, 125_000_000


@pytest.fixture(scope="module")
def ops():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gpusdr import ops
    return ops


@pytest.fixture(scope="module")
def shard(ops, orc):
    """Rank 1 of 2 at the bench's C5 size: [3 600-sample halo | 125 M-sample segment] of the synthetic
    1 Gsps stream (the halo = the tail of rank 0's segment, as the ring exchange delivers it)."""
    import torch
    from gpusdr.shard import AmChainShard, ChainShardGeometry
    g = ChainShardGeometry(1, 2, L, T, D, TA, DA)
    rf, au = orc.lowpass_taps(T, 0.04, "blackman"), orc.lowpass_taps(TA, 0.02)
    sh = AmChainShard(g, torch.from_numpy(rf).cuda(), torch.from_numpy(au).cuda(), torch.device("cuda", 0))
    ops.synth_iq_int8(0x5EED, 1e9, 1e3, 7.5e7, g.segment_start(0) - g.halo, g.halo + L, out=sh.buf)
    assert ops.kernel_policy() & ops.POLICY_I8_WS8 == 0  # the default kernel
    yield sh, rf, au
    del sh
    torch.cuda.empty_cache()


def _step(sh):
    import torch
    sh.out.fill_(float("nan"))
    sh.am.fill_(float("nan"))
    sh._bulk()
    sh._head()
    torch.cuda.synchronize()
    return sh.out.cpu().numpy().copy(), sh.am.cpu().numpy().copy()


def _js(sh, rng):
    """Every head output, both sides of each bulk block edge, ring-wrap tiles, random outputs."""
    g = sh.geom
    ha = sh.head_audio
    n_bulk = g.rf_outputs - g.head_rf
    local = _sample_audio(-(-n_bulk // TILE), g.outputs - ha, TA, DA, 0, rng)
    return np.unique(np.concatenate([np.arange(ha + 4), local + ha]))


def test_multirank_bulk_and_head_at_bench_size(ops, orc, shard):
    """The 2-rank step's bulk + head launches at L = 125 M on the 4-way kernel: ~2 000 audio outputs and
    every head output against float64 on their own windows; the bulk's AM samples equal the plain
    gsdrInt8FirFCAmDemod call's bit for bit; no hand-off abort; a repeat is bit-identical."""
    import torch
    from gpusdr import ops as o
    sh, rf, au = shard
    g = sh.geom
    assert sh.head_audio == 18 and g.head_rf == 360
    assert ops.fir_kernel_class(sh.seg, sh.rf_taps, D, int8_iq=True) == "i8-dec-mfma"  # the 4-way kernel: policy 0
    ops.ws_aborts(reset=True)
    out, am = _step(sh)
    assert ops.ws_aborts(reset=True) == 0
    assert np.all(np.isfinite(out)) and np.all(np.isfinite(am))
    js = _js(sh, np.random.default_rng(6))
    assert len(js) >= 1500
    _check_audio_sampled(orc, sh.buf, rf, au, D, DA, js, out[js])
    # the fused bulk's AM samples = the plain call over the segment (same kernel, same tiles)
    n_bulk = g.rf_outputs - g.head_rf
    am_ref = o.fir(sh.rf_taps, sh.seg, D, n_bulk, am=True, int8_iq=True)
    torch.cuda.synchronize()
    assert am[g.head_rf:].tobytes() == am_ref.cpu().numpy().tobytes()
    out2, am2 = _step(sh)
    assert out2.tobytes() == out.tobytes() and am2.tobytes() == am.tobytes()


def test_multirank_bulk_and_head_abort_path(ops, shard):
    """The same launches with every hand-off wait giving up at once (spin limit 0): the launch drains, the
    abort is counted, nothing faults (the synchronize after it succeeds), the next launch reports it
    (hipErrorLaunchTimeOut) and after the count is read the launches are exact again."""
    import torch
    from gpusdr._native import HipError
    sh, _, _ = shard
    ref, _ = _step(sh)
    prev = ops.set_ws_spin_limit(0)
    try:
        ops.ws_aborts(reset=True)
        sh._bulk()
        torch.cuda.synchronize()  # an illegal access would surface here
    finally:
        ops.set_ws_spin_limit(prev)
    assert ops.ws_aborts(reset=False) > 0
    with pytest.raises(HipError):
        sh._bulk()  # reports the pending abort, launches nothing
    assert ops.ws_aborts(reset=True) == 0  # the failed call took the count
    out, _ = _step(sh)
    assert ops.ws_aborts(reset=True) == 0
    assert out.tobytes() == ref.tobytes()


def test_multirank_step_beside_concurrent_hbm_traffic(ops, shard):
    """correct work must not fail because other work shares the GPU. Each bulk + head
    step runs while another stream copies 2 GiB (the HBM probe's copy mode) and streams a 1 GiB copy
    kernel: no abort (the hand-off budget is wall clock now, not a poll count), outputs bit-identical to
    the uncontended step."""
    import torch
    sh, _, _ = shard
    ref, ref_am = _step(sh)
    side = torch.cuda.Stream()
    src = torch.empty(1 << 31, dtype=torch.uint8, device="cuda")
    dst = torch.empty_like(src)
    ops.ws_aborts(reset=True)
    for _ in range(4):
        with torch.cuda.stream(side):
            ops.hbm_probe(src, dst, 1)
            ops.copy_kernel(dst[: 1 << 30], src[: 1 << 30])
            ops.hbm_probe(src, dst, 1)
        sh.out.fill_(float("nan"))
        sh._bulk()
        sh._head()
        torch.cuda.synchronize()
        assert ops.ws_aborts(reset=True) == 0
        assert sh.out.cpu().numpy().tobytes() == ref.tobytes()
        assert sh.am.cpu().numpy().tobytes() == ref_am.tobytes()
    del src, dst
