"""The C5 receive chain in ONE launch (gsdrInt8FirFCAmDemodFirFF: int8 IQ -> FC FIR -> AM -> FF audio
FIR, the AM samples in an LDS ring of the wave-specialised int8 MFMA kernel, the audio FIR on its
producer waves) against the float64 oracle chain, and against the two reference calls it stands for
(gsdrInt8FirFCAmDemod then gsdrFirFF over [AM history | new AM], QuadAmDemod.cpp:93-98 + Fir.cpp:229-269):
the AM samples bit for bit, the audio within the oracle bound (the audio sum runs in another order)."""
import numpy as np
import pytest

FIR_TOL = 1e-6


@pytest.fixture(scope="module")
def ops():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gpusdr import ops
    return ops


def _expected_audio(orc, am64, rf_bound, audio_taps, Da, n):
    """float64 audio FIR over the float64 AM stream + the bound: the RF FIR bound and the sqrt
    rounding carried through |audio taps|, plus the audio FIR's own bound."""
    audio, audio_bound = orc.fir_f64(audio_taps, am64.astype(np.float32), Da, n)
    carried, _ = orc.fir_f64(np.abs(audio_taps), (FIR_TOL * (rf_bound + am64)).astype(np.float32), Da, n)
    return audio, carried + FIR_TOL * audio_bound + 1e-30


def _run(ops, orc, T, D, Ta, Da, n_hist_rf, n_rf, H, seed, store=True, check_kernel=True, poison=False):
    """RF outputs [0, n_hist_rf) by the plain call (the history), then the fused call over RF outputs
    [n_hist_rf, n_hist_rf + n_rf) with the last H of the earlier AM samples as its history."""
    import torch
    rng = np.random.default_rng(seed)
    rf = orc.lowpass_taps(T, 0.4 / D, "blackman")
    au = orc.lowpass_taps(Ta, 0.4 / Da)
    n_all = n_hist_rf + n_rf
    iq = rng.integers(-128, 128, size=2 * ((n_all - 1) * D + T)).astype(np.int8)
    dev = torch.from_numpy(iq).cuda()
    rf_d, au_d = torch.from_numpy(rf).cuda(), torch.from_numpy(au).cuda()
    if check_kernel:
        assert ops.fir_kernel_class(dev, rf_d, D, int8_iq=True) == "i8-dec-mfma"
    am_all = torch.zeros(n_all, dtype=torch.float32, device="cuda")
    if n_hist_rf:
        ops.fir(rf_d, dev, D, n_hist_rf, out=am_all[:n_hist_rf], am=True, int8_iq=True)
    window = am_all[n_hist_rf - H:]
    n_audio = (H + n_rf - Ta) // Da + 1
    audio = torch.full((n_audio,), float("nan"), dtype=torch.float32, device="cuda")
    if poison:  # every CU's LDS filled with NaN just before the launch
        ops.poison_lds(0)
    ops.am_chain_fused(rf_d, dev[2 * n_hist_rf * D:], D, n_rf, window, H, au_d, Da, n_audio, audio, store_am=store)
    # the two reference calls over the same input
    am_ref = torch.empty(n_rf, dtype=torch.float32, device="cuda")
    ops.fir(rf_d, dev[2 * n_hist_rf * D:], D, n_rf, out=am_ref, am=True, int8_iq=True)
    win_ref = torch.cat([am_all[n_hist_rf - H: n_hist_rf], am_ref])
    audio_ref = ops.fir(au_d, win_ref, Da, n_audio)
    torch.cuda.synchronize()
    x = orc.int8_to_float(iq).view(np.complex64)
    y, rf_bound = orc.fir_f64(rf, x, D, n_all)
    am64 = np.abs(y)
    lo = n_hist_rf - H
    want, bound = _expected_audio(orc, am64[lo:], rf_bound[lo:], au, Da, n_audio)
    got = audio.cpu().numpy()
    ref = audio_ref.cpu().numpy()
    assert np.all(np.isfinite(got))
    assert np.all(np.abs(got - want) <= bound), np.max(np.abs(got - want) / bound)
    assert np.all(np.abs(ref - want) <= bound)
    assert np.all(np.abs(got - ref) <= 2 * bound)
    if store:  # the AM samples are the plain call's, bit for bit
        assert am_all[n_hist_rf:].cpu().numpy().tobytes() == am_ref.cpu().numpy().tobytes()
    return got


@pytest.mark.gpu
@pytest.mark.parametrize("T,D,Ta,Da,n_rf", [
    (1023, 10, 255, 20, 200_000),   # C5's filters, ~390 tiles: every block has a lead tile
    (1023, 10, 255, 20, 1_000),     # 2 tiles: blocks of one tile (lead + one)
    (1023, 10, 255, 20, 255),       # one tile, exactly one audio output
    (255, 5, 63, 8, 70_001),        # ragged last tile
    (511, 8, 256, 3, 40_000),       # 256 audio taps (the most the ring stage takes), D_a = 3
    (160, 16, 17, 64, 30_000),      # D_a > a tile's share of outputs per wave batch
    (64, 2, 9, 1, 9_000),           # D_a = 1: 57 outputs per tile per wave
])
def test_fused_chain_matches_oracle(ops, orc, T, D, Ta, Da, n_rf):
    _run(ops, orc, T, D, Ta, Da, 0, n_rf, 0, seed=T + n_rf)


@pytest.mark.gpu
@pytest.mark.parametrize("H", [1, 254, 3000])
def test_fused_chain_with_am_history(ops, orc, H):
    """History in front of the new AM samples (the chunked / resident executors' carried ra samples);
    H > Ta: the first audio windows lie wholly in the history."""
    _run(ops, orc, 1023, 10, 255, 20, 5000, 60_000, H, seed=H)


@pytest.mark.gpu
def test_fused_chain_without_am_store(ops, orc):
    """store_am = False (the sharded C5 step: nothing downstream reads the AM samples): same audio."""
    a = _run(ops, orc, 1023, 10, 255, 20, 0, 100_000, 0, seed=3, store=False)
    b = _run(ops, orc, 1023, 10, 255, 20, 0, 100_000, 0, seed=3, store=True)
    assert a.tobytes() == b.tobytes()


@pytest.mark.gpu
def test_fused_chain_fallback_shapes(ops, orc):
    """Shapes / policies the fused kernel does not take run the two calls: > 256 audio taps; the
    barrier-synchronous policy."""
    _run(ops, orc, 255, 5, 300, 4, 0, 20_000, 0, seed=7)
    prev = ops.set_kernel_policy(ops.POLICY_NO_WS)
    try:
        _run(ops, orc, 1023, 10, 255, 20, 0, 20_000, 0, seed=8, check_kernel=False)
    finally:
        ops.set_kernel_policy(prev)


@pytest.mark.gpu
def test_fused_chain_rejects_short_am(ops, orc):
    import torch
    rf = torch.from_numpy(orc.lowpass_taps(1023, 0.04)).cuda()
    au = torch.from_numpy(orc.lowpass_taps(255, 0.02)).cuda()
    iq = torch.zeros(2 * (999 * 10 + 1023), dtype=torch.int8, device="cuda")
    win = torch.empty(1000, dtype=torch.float32, device="cuda")
    out = torch.empty(100, dtype=torch.float32, device="cuda")
    with pytest.raises(ValueError):
        ops.am_chain_fused(rf, iq, 10, 1000, win, 0, au, 20, 100, out)
    from gpusdr._native import lib
    r = lib().gsdrInt8FirFCAmDemodFirFF(10, rf.data_ptr(), 1023, iq.data_ptr(), 1000, win.data_ptr(), 0, 1, 20,
                                        au.data_ptr(), 255, out.data_ptr(), 100, 0, None)
    assert r != 0


@pytest.mark.gpu
@pytest.mark.parametrize("T,D,Ta,Da", [(127, 1, 63, 4), (64, 3, 31, 5)])
def test_fused_chain_short_filters_ring_order(ops, orc, T, D, Ta, Da):
    """Short RF filters (2 K-steps per consumer wave): the consumer waves hand tiles off quickly, and
    a wave could finish tile t + 1 before a slower one had written its share of tile t - the audio
    stage waits for each ring slot it reads (per-slot counts), not for a tile count. Repeated
    launches of varying tile counts over random data, every one against the float64 oracle (AM not
    stored: at D = 1 the plain call runs another kernel, so the AM samples are not the bit-equality
    reference here)."""
    for rep in range(12):
        _run(ops, orc, T, D, Ta, Da, 0, 25_000 + 509 * rep, 0, seed=1000 * T + rep, store=False,
             check_kernel=False)


@pytest.mark.gpu
@pytest.mark.parametrize("ws8", [False, True])
@pytest.mark.parametrize("T,D,Ta,Da,n_rf", [(64, 3, 31, 5, 1000), (127, 1, 63, 4, 1500), (1023, 10, 255, 20, 1000),
                                            (1023, 10, 255, 20, 300_000)])
def test_fused_chain_ignores_stale_lds(ops, orc, T, D, Ta, Da, n_rf, ws8):
    """LDS poisoned with NaN right before each launch: nothing the kernel did not write may reach an
    output. The audio windows read 256 AM-ring samples and multiply those past their taps by zero
    (0 * NaN = NaN), so ring slots a block never fills must hold zeros - r04 found NaN audio in
    short-filter steps on fresh boxes before the ring was zeroed per launch. Both int8 kernels: the
    default 4-way one and the r04 8-way one (GSDR_POLICY_I8_WS8)."""
    prev = ops.set_kernel_policy(ops.POLICY_I8_WS8 if ws8 else 0)
    try:
        for rep in range(4):
            _run(ops, orc, T, D, Ta, Da, 0, n_rf + 37 * rep, 0, seed=17 * T + rep, store=False, check_kernel=False,
                 poison=True)
    finally:
        ops.set_kernel_policy(prev)


# ---- the fused kernel at the sizes it is timed at (VERDICT r04 missing 1) ---------------------------

TILE = 512     # RF outputs per tile (kCfTileOut)
BLOCKS = 256   # the launcher's grid: min(tiles, 256) blocks, each a contiguous tile range
RING = 8       # AM ring slots (kAmRing): a block reuses a slot from its 9th tile (lead included) on


def _block_ranges(tiles):
    """(first tile, tile count) of every block as the kernel splits them, the lead tile (the one in front
    of every block but the first, computed into its ring only) included."""
    grid = min(tiles, BLOCKS)
    q, r = divmod(tiles, grid)
    out = []
    for b in range(grid):
        t0, n = b * q + min(b, r), q + (1 if b < r else 0)
        if t0 > 0:
            t0, n = t0 - 1, n + 1
        out.append((t0, n))
    return out


def _sample_audio(tiles, n_audio, Ta, Da, amH, rng, n_random=500, wrap_blocks=32):
    """Audio outputs to check: the first and last output owned by every block (the outputs on both sides
    of each block-range edge), the outputs of the tiles around every ring wrap (block-local tiles 7-9,
    15-17 and the last two) of `wrap_blocks` blocks, and random ones. Output j is owned by the tile holding
    its window's last AM sample j Da - amH + Ta - 1."""
    def owned(t):  # audio outputs whose window ends in tile t
        lo = max(0, -(-(t * TILE - Ta + 1 + amH) // Da))
        hi = min(n_audio, -(-((t + 1) * TILE - Ta + 1 + amH) // Da))
        return lo, hi
    ranges = _block_ranges(tiles)
    picks = []
    for b, (t0, n) in enumerate(ranges):
        first = t0 + (1 if t0 > 0 else 0)  # the block's own first tile (after the lead)
        lo, _ = owned(first)
        _, hi = owned(t0 + n - 1)
        picks += [lo, hi - 1]
    for b in rng.choice(len(ranges), size=min(wrap_blocks, len(ranges)), replace=False):
        t0, n = ranges[b]
        for loc in (7, 8, 9, 15, 16, 17, n - 2, n - 1):
            if 0 <= loc < n:
                lo, hi = owned(t0 + loc)
                if hi > lo:
                    picks += [lo, (lo + hi) // 2, hi - 1]
    picks += list(rng.integers(0, n_audio, n_random))
    js = np.unique(np.asarray(picks, dtype=np.int64))
    return js[(js >= 0) & (js < n_audio)]


def _check_audio_sampled(orc, iq_dev, rf, au, D, Da, js, got):
    """Audio outputs js of a fused launch over iq_dev (AM history none: audio j reads RF outputs
    [j Da, j Da + Ta), RF output k reads input samples [k D, k D + T)) against float64 on their own input
    windows gathered on the GPU; the bound as _expected_audio's."""
    import torch
    T, Ta = len(rf), len(au)
    span = (Ta - 1) * D + T
    idx = torch.from_numpy(2 * js * Da * D).cuda()[:, None] + torch.arange(2 * span, device="cuda")[None, :]
    w = orc.int8_to_float(iq_dev[idx].cpu().numpy().reshape(-1)).view(np.complex64).reshape(len(js), span)
    bad = []
    for r, j in enumerate(js):
        y, rf_bound = orc.fir_f64(rf, w[r], D, Ta)
        a = np.abs(y)
        want, audio_bound = orc.fir_f64(au, a.astype(np.float32), Da, 1)
        carried, _ = orc.fir_f64(np.abs(au), (FIR_TOL * (rf_bound + a)).astype(np.float32), Da, 1)
        if not abs(got[r] - want[0]) <= carried[0] + FIR_TOL * audio_bound[0] + 1e-30:
            bad.append((int(j), float(got[r]), float(want[0])))
    assert not bad, f"{len(bad)} of {len(js)} sampled audio outputs outside the bound: {bad[:8]}"


@pytest.mark.gpu
def test_fused_chain_full_c5_size(ops, orc):
    """The bench's exact N = 1 C5 step (AmChainShard.step over [3 600-sample cascaded halo | 125 M int8 IQ
    samples], store_am = False: ONE gsdrInt8FirFCAmDemodFirFF launch of 12.5 M RF outputs = 24 415 tiles,
    ~96 per block, so every block's 8-slot AM ring wraps ~12 times behind the amFree hand-off): ~2 000
    audio outputs - both sides of every block-range edge, the tiles around ring wraps, random ones -
    against float64 on their own windows gathered on the GPU. Reference chain: am_test.cpp:352-433,
    QuadAmDemod.cpp:93-98, Fir.cpp:229-269."""
    import torch
    from gpusdr.shard import AmChainShard, ChainShardGeometry
    T, D, Ta, Da, L = 1023, 10, 255, 20, 125_000_000
    g = ChainShardGeometry(0, 1, L, T, D, Ta, Da)
    rf, au = orc.lowpass_taps(T, 0.04, "blackman"), orc.lowpass_taps(Ta, 0.02)
    sh = AmChainShard(g, torch.from_numpy(rf).cuda(), torch.from_numpy(au).cuda(), torch.device("cuda", 0))
    ops.synth_iq_int8(0x5EED, 1e9, 1e3, 7.5e7, 0, g.halo + L, out=sh.buf)
    assert ops.fir_kernel_class(sh.buf, sh.rf_taps, D, int8_iq=True) == "i8-dec-mfma"
    ops.ws_aborts(reset=True)
    out = sh.step(carry=False)
    torch.cuda.synchronize()
    assert ops.ws_aborts(reset=True) == 0
    tiles = -(-g.rf_outputs // TILE)
    assert tiles // BLOCKS + 1 > 9 * RING  # the ring wraps many times in every block
    got_all = out.cpu().numpy()
    assert len(got_all) == g.outputs and np.all(np.isfinite(got_all))
    js = _sample_audio(tiles, g.outputs, Ta, Da, 0, np.random.default_rng(125))
    assert len(js) >= 1500
    _check_audio_sampled(orc, sh.buf, rf, au, D, Da, js, got_all[js])
    # the r04 8-way kernel (GSDR_POLICY_I8_WS8) at the same size: its ring wrap under test too
    prev = ops.set_kernel_policy(ops.POLICY_I8_WS8)
    try:
        out8 = sh.step(carry=False).cpu().numpy()
    finally:
        ops.set_kernel_policy(prev)
    assert ops.ws_aborts(reset=True) == 0 and np.all(np.isfinite(out8))
    _check_audio_sampled(orc, sh.buf, rf, au, D, Da, js, out8[js])
    del sh
    torch.cuda.empty_cache()


@pytest.mark.gpu
@pytest.mark.parametrize("tiles_per_block,poison", [(9, False), (13, True), (20, False)])
def test_fused_chain_mid_size_c5_filters(ops, orc, tiles_per_block, poison):
    """C5's filters at 9-20 tiles per block (the ring wraps once or twice per block; VERDICT r04 asks for
    this range), LDS poisoned with NaN before the launch in one case: sampled float64 check as above,
    plus the AM samples bit for bit against the plain gsdrInt8FirFCAmDemod call."""
    import torch
    T, D, Ta, Da = 1023, 10, 255, 20
    n_rf = BLOCKS * TILE * tiles_per_block - 77  # a ragged last tile
    n_in = (n_rf - 1) * D + T
    rf, au = orc.lowpass_taps(T, 0.04, "blackman"), orc.lowpass_taps(Ta, 0.02)
    rf_d, au_d = torch.from_numpy(rf).cuda(), torch.from_numpy(au).cuda()
    iq = ops.synth_iq_int8(0x5EED, 1e9, 1e3, 7.5e7, 123_456 * tiles_per_block, n_in)
    n_audio = (n_rf - Ta) // Da + 1
    am = torch.zeros(n_rf, dtype=torch.float32, device="cuda")
    audio = torch.full((n_audio,), float("nan"), dtype=torch.float32, device="cuda")
    if poison:
        ops.poison_lds(0)
    ops.am_chain_fused(rf_d, iq, D, n_rf, am, 0, au_d, Da, n_audio, audio, store_am=True)
    am_ref = ops.fir(rf_d, iq, D, n_rf, am=True, int8_iq=True)
    torch.cuda.synchronize()
    assert torch.equal(am, am_ref)
    got_all = audio.cpu().numpy()
    assert np.all(np.isfinite(got_all))
    tiles = -(-n_rf // TILE)
    js = _sample_audio(tiles, n_audio, Ta, Da, 0, np.random.default_rng(tiles_per_block), n_random=300)
    _check_audio_sampled(orc, iq, rf, au, D, Da, js, got_all[js])


@pytest.mark.gpu
@pytest.mark.parametrize("T,D,Ta,Da,tiles_per_block", [(127, 1, 63, 4, 10), (64, 3, 31, 5, 17), (255, 5, 63, 8, 12)])
def test_fused_chain_mid_size_short_filters(ops, orc, T, D, Ta, Da, tiles_per_block):
    """Short RF filters (2-4 K-steps per consumer wave: the fastest hand-offs, the amFree / amSlot
    protocol under the most pressure) at 10-17 tiles per block, so the 8-slot ring wraps inside every
    block; LDS poisoned before each launch; the whole audio stream against the float64 oracle chain."""
    for rep in range(2):
        n_rf = BLOCKS * TILE * tiles_per_block - 131 * rep
        _run(ops, orc, T, D, Ta, Da, 0, n_rf, 0, seed=31 * T + rep, store=False, check_kernel=False,
             poison=True)
