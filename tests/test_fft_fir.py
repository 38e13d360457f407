"""GPU parity of the FFT fast-convolution FIR (cuda-sdr_amd/csrc/kernels/fir_fft.hip).

The long real-tap FC FIRs (T >= 256, D in {2, 4, 6, 8, 10}; C3 and the C5 RF stage) run as a
polyphase overlap-save FFT. Same contract and tolerance as every FIR path
(tests/test_gpu_parity.py): per element |y - y64| <= 1e-6 * sum_j |h_j||x_kD+j| against the
float64 oracle (y[k] = sum_j h[j] x[kD + j], src/filters/Fir.cpp:229-269), relative L2 <= 1e-6.
The accuracy guard (blocks whose row levels spread more than the guard ratio take the direct
form) is exercised with bursts, silence, ramps, impulses and inf/NaN samples, and the tests check
through the fallback counter that ordinary data really runs on the FFT.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIR_TOL = 1e-6


@pytest.fixture(scope="module")
def ops():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gpusdr import ops as _ops
    return _ops


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


def _check(y, y64, bound, what):
    """Per element against the window's own scale; relative L2 where the output is passband-
    dominated (||y64|| >= 0.1 ||sum|h||x|||). A stopband-only output (e.g. a carrier the low-pass
    rejects) is ~1e-3 of its inputs' level, so its relative L2 measures the fp32 floor of ANY
    float32 form (the direct form included), not this kernel; the per-element bound still holds."""
    err = np.abs(y.astype(np.complex128) - y64)
    worst = float(np.max(err / (bound + 1e-300)))
    assert np.all(err <= FIR_TOL * bound + 1e-30), (what, worst)
    den = np.linalg.norm(y64)
    if den > 0 and den >= 0.1 * np.linalg.norm(bound):
        rel = float(np.linalg.norm(y - y64) / den)
        assert rel <= FIR_TOL, (what, rel, worst, int(np.argmax(err / (bound + 1e-300))), len(y))
    return worst


def _signal(kind, n, seed, orc):
    rng = np.random.default_rng(seed)
    if kind == "c64":
        return orc.synth_wideband_cf32(0xC3 + seed, 0.013, 0.31, 1000 * seed, n)
    if kind == "c64-noise":
        return (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
    return orc.synth_iq_int8(0x5EED + seed, 1e9, 1e3, 7.5e7, 1000 * seed, n)


FFT_CASES = [("c64", 1023, 10, 20000), ("c64", 1023, 10, 1), ("c64", 1023, 10, 410), ("c64", 1023, 10, 411),
             ("c64-noise", 1023, 10, 30000), ("c64", 256, 2, 5000), ("c64-noise", 511, 4, 7777),
             ("c64", 600, 6, 3001), ("c64-noise", 2000, 8, 4096), ("c64", 4000, 10, 999),
             ("i8", 1023, 10, 20000), ("i8", 1023, 10, 1), ("i8", 300, 2, 5000), ("i8", 700, 4, 12345),
             ("i8", 1000, 8, 2222),
             # D = 1 (firFftD1Kernel: 8 output phases of 512 - ceil(T/8) rows per block)
             ("c64", 1023, 1, 20000), ("c64", 1023, 1, 1), ("c64", 1023, 1, 3072), ("c64", 1023, 1, 3073),
             ("c64-noise", 256, 1, 9999), ("c64", 3584, 1, 5000), ("c64-noise", 2000, 1, 7001)]


@pytest.mark.parametrize("kind,T,D,n_out", FFT_CASES)
def test_fft_fir_matches_float64(ops, orc, kind, T, D, n_out):
    n_in = (n_out - 1) * D + T
    x = _signal(kind, n_in, T + D, orc)
    taps = orc.lowpass_taps(T, 0.4 / D).astype(np.float32)
    taps[T // 3] *= -1.5
    i8 = kind == "i8"
    x_d, taps_d = _dev(x), _dev(taps)
    ops.fft_direct_blocks(reset=True)
    with _Policy(ops, ops.POLICY_PREFER_FFT):  # int8: the FFT even where the int8 MFMA kernels apply
        assert ops.fir_kernel_class(x_d, taps_d, D, int8_iq=i8) == "fft"
        y = _host(ops.fir(taps_d, x_d, D, n_out, int8_iq=i8))
        am = _host(ops.fir(taps_d, x_d, D, n_out, int8_iq=i8, am=True))
    direct = ops.fft_direct_blocks(reset=True)
    xc = orc.int8_to_float(x).view(np.complex64) if i8 else x
    y64, bound = orc.fir_f64(taps, xc, D, n_out)
    _check(y, y64, bound, ("fft", kind, T, D, n_out))
    assert np.all(np.abs(am - np.abs(y64)) <= FIR_TOL * bound + 1e-30), ("fft-am", kind, T, D)
    # ordinary signals run on the FFT (at most the final, partly-zero block may take the direct form)
    blocks = -(-n_out // (512 - -(-T // D) + 1))
    assert direct <= 2, (direct, blocks)


CC_CASES = [(1023, 10, 20000), (1023, 10, 1), (600, 6, 3001), (256, 2, 5000), (2000, 8, 999),
            (1023, 1, 20000), (1023, 1, 3073), (256, 1, 777)]


@pytest.mark.parametrize("T,D,n_out", CC_CASES)
def test_fft_fir_complex_taps(ops, orc, T, D, n_out):
    """gsdrFirCC / gsdrFirCCAmDemod (Fir.cpp:250-258, complex taps, non-conjugate MAC - SURVEY 8(c))
    on the FFT kernels: the filter spectra are complex anyway, G_p = conj(DFT(conj h_p)) / M. A
    complex band-pass (a low-pass shifted by exp(j 2 pi f0 j)) against float64, complex and AM
    outputs, ordinary data on the FFT (no direct-form blocks), and the direct-form fallback (guard 0)
    within the same bound."""
    n_in = (n_out - 1) * D + T
    x = _signal("c64-noise" if T % 2 else "c64", n_in, T + 3 * D, orc)
    j = np.arange(T)
    taps = (orc.lowpass_taps(T, 0.4 / D).astype(np.float64) * np.exp(2j * np.pi * 0.11 / D * j)).astype(np.complex64)
    taps[T // 3] *= -1.5 + 0.5j
    x_d, taps_d = _dev(x), _dev(taps)
    ops.fft_direct_blocks(reset=True)
    y = _host(ops.fir(taps_d, x_d, D, n_out))
    am = _host(ops.fir(taps_d, x_d, D, n_out, am=True))
    assert ops.fft_direct_blocks(reset=True) <= 2
    y64, bound = orc.fir_f64(taps, x, D, n_out)
    _check(y, y64, bound, ("fft-cc", T, D, n_out))
    assert np.all(np.abs(am - np.abs(y64)) <= FIR_TOL * bound + 1e-30), ("fft-cc-am", T, D)
    prev = ops.set_fft_guard(0.0)  # every block in the direct form
    try:
        yd = _host(ops.fir(taps_d, x_d, D, n_out))
        assert ops.fft_direct_blocks(reset=True) > 0
    finally:
        ops.set_fft_guard(prev)
    _check(yd, y64, bound, ("fft-cc-direct", T, D, n_out))


def test_fft_fir_large_stream_properties(ops, orc):
    """2^24-sample C3-shaped stream: a sampled float64 check across the whole range, and the
    FFT result equals the direct forms (MFMA and fp32 VALU kernels) within the same tolerance."""
    T, D = 1023, 10
    n_in = 1 << 24
    n_out = (n_in - T) // D + 1
    x_d = ops.synth_wideband_cf32(0xC3, 0.013, 0.31, 0, n_in)
    taps = orc.lowpass_taps(T, 0.04, "blackman")
    taps_d = _dev(taps)
    with _Policy(ops, ops.POLICY_PREFER_FFT):  # below 2^24 input samples cf32 takes the MFMA kernel by default
        am = _host(ops.fir(taps_d, x_d, D, n_out, am=True))
    x = _host(x_d)
    rng = np.random.default_rng(3)
    ks = np.unique(np.concatenate([rng.integers(0, n_out, 3000), [0, n_out - 1]]))
    for k in ks[::50]:
        y64, bound = orc.fir_f64(taps, x[k * D: k * D + T], D, 1)
        assert abs(am[k] - abs(y64[0])) <= FIR_TOL * bound[0], k
    with _Policy(ops, ops.POLICY_NO_FFT):
        am_mfma = _host(ops.fir(taps_d, x_d, D, n_out, am=True))
    # both within 1e-6 sum|h||x| of float64 => within 2e-6 of each other; sum|h||x| >= 0.45 sum|h|
    # for this signal (|x| >= 1 - 0.5 - 0.02)
    assert np.max(np.abs(am - am_mfma)) <= 2 * FIR_TOL * 0.45 * np.abs(taps).sum() * 1.01


def test_fft_fir_full_c3_size(ops, orc):
    """BASELINE's C3 at full size (2^28 - 6 cf32 samples, 1023 taps, D = 10, AM): 4 000 outputs
    sampled over the whole stream - the first and last, both sides of FFT block boundaries and
    random ones - against float64 on their own windows (gathered on the GPU), and no block took the
    direct-form fallback on this signal."""
    import torch
    T, D = 1023, 10
    n_in = (1 << 28) - (1 << 28) % D
    n_out = (n_in - T) // D + 1
    x_d = ops.synth_wideband_cf32(0xC3, 0.013, 0.31, 0, n_in)
    taps = orc.lowpass_taps(T, 0.04, "blackman")
    ops.fft_direct_blocks(0, reset=True)
    am = ops.fir(_dev(taps), x_d, D, n_out, am=True)
    torch.cuda.synchronize()
    assert ops.fft_direct_blocks(0, reset=True) == 0
    rng = np.random.default_rng(28)
    V = 512 - (T + D - 1) // D + 1  # outputs per FFT block
    edges = np.arange(V, n_out, V * 977)
    ks = np.unique(np.concatenate([[0, 1, n_out - 2, n_out - 1], edges - 1, edges,
                                   rng.integers(0, n_out, 4000 - 2 * len(edges) - 4)]))
    ks = ks[ks < n_out]
    idx = torch.from_numpy(ks * D).cuda()[:, None] + torch.arange(T, device="cuda")[None, :]
    windows = x_d[idx].cpu().numpy()          # (len(ks), T) complex64
    got = am[torch.from_numpy(ks).cuda()].cpu().numpy()
    y = windows.astype(np.complex128) @ taps.astype(np.float64)
    bound = np.abs(windows).astype(np.float64) @ np.abs(taps.astype(np.float64))
    err = np.abs(got - np.abs(y))
    assert np.all(err <= FIR_TOL * bound), float(np.max(err / bound))


@pytest.mark.parametrize("log2n,am", [(30, True), (27, False)])
def test_fft_fir_full_c4_size(ops, orc, log2n, am):
    """BASELINE's C4 at full size on the D = 1 kernel (firFftD1PfKernel): the bench's c4s launch
    (2^30 cf32 samples = 8 GiB in, 1023 taps, AM: 4 GiB out) and a 2^27-sample complex-output launch.
    Block b covers outputs [b 8V, (b + 1) 8V), V = 512 - ceil(T / 8) = 384 rows, so 3 072 outputs per
    block: 4 000 outputs - first and last, both sides of block edges spread over the stream (past 2^31
    bytes of input and of output, where a 32-bit row or byte index would wrap), the eight output phases
    of a row and random ones - against float64 on their own windows gathered on the GPU; no block took
    the direct-form fallback."""
    import torch
    T, D = 1023, 1
    n_in = 1 << log2n
    n_out = n_in - T + 1
    x_d = ops.synth_wideband_cf32(0xC4, 0.013, 0.31, 0, n_in)
    taps = orc.lowpass_taps(T, 0.04, "blackman")
    taps_d = _dev(taps)
    assert ops.fir_kernel_class(x_d, taps_d, D) == "fft"
    ops.fft_direct_blocks(0, reset=True)
    y_d = ops.fir(taps_d, x_d, D, n_out, am=am)
    torch.cuda.synchronize()
    assert ops.fft_direct_blocks(0, reset=True) == 0
    rng = np.random.default_rng(log2n)
    per_block = 8 * (512 - -(-T // 8))
    edges = np.arange(per_block, n_out, per_block * 4099)
    rows = rng.integers(0, n_out // 8, 16) * 8
    ks = np.unique(np.concatenate([[0, 1, 7, 8, n_out - 2, n_out - 1], edges - 1, edges,
                                   (rows[:, None] + np.arange(8)[None, :]).ravel(),
                                   rng.integers(0, n_out, 4000 - 2 * len(edges) - 134)]))
    ks = ks[ks < n_out]
    assert ks.max() * 8 > 1 << 31 or log2n < 28
    idx = torch.from_numpy(ks).cuda()[:, None] + torch.arange(T, device="cuda")[None, :]
    windows = x_d[idx].cpu().numpy()
    got = y_d[torch.from_numpy(ks).cuda()].cpu().numpy()
    y = windows.astype(np.complex128) @ taps.astype(np.float64)
    bound = np.abs(windows).astype(np.float64) @ np.abs(taps.astype(np.float64))
    err = np.abs(got - (np.abs(y) if am else y))
    assert np.all(err <= FIR_TOL * bound), float(np.max(err / bound))
    del x_d, y_d
    torch.cuda.empty_cache()


class _Policy:
    def __init__(self, ops, flags):
        self.ops, self.flags = ops, flags

    def __enter__(self):
        self.prev = self.ops.set_kernel_policy(self.flags)

    def __exit__(self, *exc):
        self.ops.set_kernel_policy(self.prev)


def _adversarial(name, n, rng):
    x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
    i = np.arange(n)
    if name == "bursts":
        x *= np.where((i // 3000) % 2 == 0, 1.0, 1e-6).astype(np.float32)
    elif name == "silence":
        x[(i // 7000) % 3 == 1] = 0
    elif name == "ramp":
        x *= np.exp(np.linspace(0, np.log(1e5), n)).astype(np.float32)
    elif name == "impulses":
        x = np.zeros(n, np.complex64)
        x[::997] = 1 + 1j
    elif name == "am-deep":
        x *= (1.0 + 0.999 * np.cos(2 * np.pi * i / 40000)).astype(np.float32)
    return x


@pytest.mark.parametrize("name", ["bursts", "silence", "ramp", "impulses", "am-deep"])
def test_fft_fir_guard_keeps_tolerance(ops, orc, name):
    T, D, n_out = 1023, 10, 40000
    n_in = (n_out - 1) * D + T
    x = _adversarial(name, n_in, np.random.default_rng(11))
    taps = orc.lowpass_taps(T, 0.04, "blackman")
    y = _host(ops.fir(_dev(taps), _dev(x), D, n_out))
    y64, bound = orc.fir_f64(taps, x, D, n_out)
    _check(y, y64, bound, ("guard", name))


def test_fft_fir_nonfinite_stays_local(ops, orc):
    """An inf / NaN sample poisons only the outputs whose window holds it (direct-form blocks)."""
    T, D, n_out = 1023, 10, 20000
    n_in = (n_out - 1) * D + T
    x = orc.synth_wideband_cf32(7, 0.013, 0.31, 0, n_in)
    x[50_000] = np.inf
    x[120_003] = np.nan
    taps = orc.lowpass_taps(T, 0.04, "blackman")
    y = _host(ops.fir(_dev(taps), _dev(x), D, n_out))
    k = np.arange(n_out)
    bad = np.zeros(n_out, bool)
    for pos in (50_000, 120_003):
        bad |= (k * D <= pos) & (pos < k * D + T)
    assert np.all(np.isfinite(y[~bad]))
    y64, bound = orc.fir_f64(taps, x, D, n_out)
    _check(y[~bad], y64[~bad], bound[~bad], "nonfinite")


@pytest.mark.parametrize("D,per_block", [(10, 410), (1, 8 * 384)])
def test_fft_fir_guard_zero_is_direct(ops, orc, D, per_block):
    """Guard ratio 0 forces every block into the direct form (the fallback path in isolation)."""
    T, n_out = 1023, 5000
    n_in = (n_out - 1) * D + T
    x = _signal("c64", n_in, 1, orc)
    taps = orc.lowpass_taps(T, 0.04, "blackman")
    prev = ops.set_fft_guard(0.0)
    try:
        ops.fft_direct_blocks(reset=True)
        with _Policy(ops, ops.POLICY_PREFER_FFT):
            y = _host(ops.fir(_dev(taps), _dev(x), D, n_out))
        direct = ops.fft_direct_blocks(reset=True)
    finally:
        ops.set_fft_guard(prev)
    assert direct == -(-n_out // per_block)
    y64, bound = orc.fir_f64(taps, x, D, n_out)
    _check(y, y64, bound, "guard0")


@pytest.mark.parametrize("off", [4, 8, 12])
def test_fft_fir_int8_alignment(ops, orc, off):
    """int8 IQ input at every 4-byte misalignment of a 16-byte unit (block images read at an offset)."""
    T, D, n_out = 1023, 10, 9000
    n_in = (n_out - 1) * D + T
    iq = _signal("i8", n_in + 8, 2, orc)
    x_d = _dev(iq)[off:]
    taps = orc.lowpass_taps(T, 0.04, "blackman")
    with _Policy(ops, ops.POLICY_PREFER_FFT):
        y = _host(ops.fir(_dev(taps), x_d, D, n_out, int8_iq=True))
    xc = orc.int8_to_float(iq[off:]).view(np.complex64)
    y64, bound = orc.fir_f64(taps, xc, D, n_out)
    _check(y, y64, bound, ("i8-align", off))


def test_full_c2_and_c5_sizes(ops, orc):
    """BASELINE's C2 (20 M int8 IQ, 127 taps, D = 1, AM; one launch with the history carry) and the
    C5 RF + audio chain at full size (125 M int8 IQ, 1023 taps D = 10 -> AM -> 255 taps D = 20):
    sampled outputs against float64 on their own windows gathered on the GPU."""
    import torch
    rng = np.random.default_rng(25)
    # C2
    T, D, n = 127, 1, 20_000_000
    iq = ops.synth_iq_int8(0x5EED, 20e6, 1e3, 1.5e6, 0, n + T - 1)
    taps = orc.lowpass_taps(T, 0.1)
    am = torch.empty(n, dtype=torch.float32, device="cuda")
    carry = torch.empty(2 * (T - 1), dtype=torch.int8, device="cuda")
    ops.fir_am_i8_carry(_dev(taps), iq, D, n, am, carry)
    ks = np.unique(np.concatenate([[0, n - 1], rng.integers(0, n, 3000)]))
    idx = (torch.from_numpy(2 * ks).cuda()[:, None] + torch.arange(2 * T, device="cuda")[None, :])
    w = orc.int8_to_float(iq[idx].cpu().numpy().reshape(-1)).view(np.complex64).reshape(len(ks), T)
    y = w.astype(np.complex128) @ taps.astype(np.float64)
    bound = np.abs(w).astype(np.float64) @ np.abs(taps.astype(np.float64))
    assert np.all(np.abs(am[torch.from_numpy(ks).cuda()].cpu().numpy() - np.abs(y)) <= FIR_TOL * bound)
    assert torch.equal(carry, iq[2 * n: 2 * (n + T - 1)])  # the next call's history
    # C5
    T, D, Ta, Da, n_in = 1023, 10, 255, 20, 125_000_000
    iq = ops.synth_iq_int8(0x5EED, 1e9, 1e3, 7.5e7, 0, n_in)
    rf, au = orc.lowpass_taps(T, 0.04, "blackman"), orc.lowpass_taps(Ta, 0.02)
    n_rf = (n_in - T) // D + 1
    amd = ops.fir(_dev(rf), iq, D, n_rf, am=True, int8_iq=True)
    n_au = (n_rf - Ta) // Da + 1
    aud = ops.fir(_dev(au), amd, Da, n_au)
    ks = np.unique(np.concatenate([[0, n_au - 1], rng.integers(0, n_au, 300)]))
    span = (Ta - 1) * D + T  # input samples under one audio output
    idx = (torch.from_numpy(2 * ks * Da * D).cuda()[:, None] + torch.arange(2 * span, device="cuda")[None, :])
    w = orc.int8_to_float(iq[idx].cpu().numpy().reshape(-1)).view(np.complex64).reshape(len(ks), span)
    got = aud[torch.from_numpy(ks).cuda()].cpu().numpy()
    for r, k in enumerate(ks):
        y, rf_bound = orc.fir_f64(rf, w[r], D, Ta)
        a = np.abs(y)
        want, audio_bound = orc.fir_f64(au, a.astype(np.float32), Da, 1)
        carried, _ = orc.fir_f64(np.abs(au), (FIR_TOL * (rf_bound + a)).astype(np.float32), Da, 1)
        assert abs(got[r] - want[0]) <= carried[0] + FIR_TOL * audio_bound[0] + 1e-30, k


@pytest.mark.parametrize("am", [True, False])
def test_fft_fir_d1_unaligned_output(ops, orc, am):
    """The D = 1 kernel stores a row's eight phases as 16-byte units only when `out` is 16-byte
    aligned; at an offset of one output it falls back to per-output stores: same values, nothing
    written outside the requested outputs."""
    import torch
    T, D, n_out = 1023, 1, 7001
    n_in = (n_out - 1) * D + T
    x = _signal("c64", n_in, T + D, orc)
    taps = orc.lowpass_taps(T, 0.02).astype(np.float32)
    x_d, taps_d = _dev(x), _dev(taps)
    dt = torch.float32 if am else torch.complex64
    ref = ops.fir(taps_d, x_d, D, n_out, am=am)
    buf = torch.full((n_out + 2,), 7.0, dtype=dt, device=x_d.device)
    ops.fir(taps_d, x_d, D, n_out, out=buf[1:n_out + 1], am=am)
    got = _host(buf)
    assert got[0] == 7.0 and got[-1] == 7.0
    assert np.array_equal(got[1:n_out + 1], _host(ref))
