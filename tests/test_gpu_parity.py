"""GPU parity: the gfx950 kernels (through the gsdr C-ABI) against the CPU oracle.

Tolerances (BASELINE.json north star):
  * FIR / FIR->AM: per element |y - y64| <= 1e-6 * sum_j |h_j||x_kD+j| (the float64 oracle's
    bound), plus relative L2 <= 1e-6.
  * int8 -> float and the AM envelope: bit-exact against the oracle's identical expression.
  * fused chains: bit-exact against the unfused chain of reference entry points.
"""
import os

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


class _Policy:
    """with _Policy(ops, flags): run a block under a kernel-selection policy."""

    def __init__(self, ops, flags):
        self.ops, self.flags = ops, flags

    def __enter__(self):
        self.prev = self.ops.set_kernel_policy(self.flags)

    def __exit__(self, *exc):
        self.ops.set_kernel_policy(self.prev)


def _check_fir(y, y64, bound, what, l2=True):
    err = np.abs(y.astype(np.complex128) - y64)
    assert np.all(err <= FIR_TOL * bound + 1e-30), (what, float(np.max(err / (bound + 1e-30))))
    den = np.linalg.norm(y64)
    if den > 0 and l2:
        assert np.linalg.norm(y - y64) / den <= FIR_TOL, what


def test_fir_golden_all_variants(ops, golden_dir):
    g = np.load(os.path.join(golden_dir, "fir_golden.npz"))
    keys = sorted({k.rsplit("_", 1)[0] for k in g.files})
    for key in keys:
        D = int(key.split("_D")[1])
        taps, x, y64, bound = g[key + "_taps"], g[key + "_x"], g[key + "_y"], g[key + "_bound"]
        y = _host(ops.fir(_dev(taps), _dev(x), D, len(y64)))
        _check_fir(y, y64, bound, key)


def test_fir_kats(ops):
    # FirTests.cpp:81-84 and :196-202 (full reads; chunked reads are in test_filter_graph)
    x = np.array([0.1 + 0.2j, 0.3 + 0.4j, 0.5 + 0.6j, 0.7 + 0.8j, 0.9 + 0.9j], dtype=np.complex64)
    y = _host(ops.fir(_dev(np.array([0.5, 1.0], np.float32)), _dev(x), 2))
    assert np.allclose(y, [0.35 + 0.5j, 0.95 + 1.1j], atol=1e-6)
    x = np.array([0.1 + 0.2j, 0.3 + 0.4j, 0.5 + 0.6j, 0.7 + 0.8j] * 2, dtype=np.complex64)
    y = _host(ops.fir(_dev(np.array([0.5, 1.0, 0.25], np.float32)), _dev(x), 2))
    assert np.allclose(y, [0.475 + 0.65j, 0.975 + 1.15j, 0.475 + 0.65j], atol=1e-6)


RAGGED = [
    # (T, D, nOut)
    (1, 1, 1), (2, 2, 2), (3, 2, 7), (8, 1, 511), (9, 1, 513), (63, 1, 2047), (127, 1, 2049),
    (127, 3, 1000), (1023, 10, 1537), (1023, 1, 4099), (17, 64, 300), (3, 16, 100), (2000, 7, 777),
    (4096, 1, 3000), (20000, 10, 300),  # the last one exceeds LDS: direct fallback kernel
]


@pytest.mark.parametrize("T,D,n_out", RAGGED)
@pytest.mark.parametrize("mode", ["FF", "FC", "CC", "CF"])
def test_fir_ragged(ops, orc, T, D, n_out, mode):
    rng = np.random.default_rng(T * 131 + D * 7 + n_out)
    n_in = (n_out - 1) * D + T
    taps = (rng.standard_normal(T) / np.sqrt(T)).astype(np.float32)
    if mode[0] == "C":
        taps = (taps + 1j * rng.standard_normal(T) / np.sqrt(T)).astype(np.complex64)
    if mode[1] == "C":
        x = (rng.standard_normal(n_in) + 1j * rng.standard_normal(n_in)).astype(np.complex64)
    else:
        x = rng.standard_normal(n_in).astype(np.float32)
    y64, bound = orc.fir_f64(taps, x, D, n_out)
    y = _host(ops.fir(_dev(taps), _dev(x), D, n_out))
    _check_fir(y, y64, bound, (mode, T, D, n_out))


def test_fir_misaligned_pointers(ops, orc):
    import torch
    rng = np.random.default_rng(11)
    T, D, n_out = 127, 2, 3001
    taps = rng.standard_normal(T).astype(np.float32)
    x = (rng.standard_normal((n_out - 1) * D + T + 3) + 1j * rng.standard_normal((n_out - 1) * D + T + 3))
    x = x.astype(np.complex64)
    xd = _dev(x)
    out = torch.zeros(n_out + 3, dtype=torch.complex64, device="cuda")
    for off in (1, 3):
        ops.fir(_dev(taps), xd[off:], D, n_out, out=out[off:off + n_out])
        y64, bound = orc.fir_f64(taps, x[off:], D, n_out)
        _check_fir(_host(out)[off:off + n_out], y64, bound, off)


def test_fir_does_not_write_past_outputs(ops):
    import torch
    T, D, n_out = 63, 1, 777
    x = torch.randn(n_out - 1 + T, dtype=torch.complex64, device="cuda")
    taps = torch.randn(T, device="cuda")
    out = torch.full((n_out + 1000,), 7.0 + 7.0j, dtype=torch.complex64, device="cuda")
    ops.fir(taps, x, D, n_out, out=out[:n_out])
    tail = _host(out)[n_out:]
    assert np.all(tail == np.complex64(7 + 7j))


def test_fir_inf_sample_stays_local(ops, orc):
    """A non-finite sample may only reach outputs whose taps touch it (no zero-padded tap x inf)."""
    T, D, n_out = 100, 3, 400
    x = np.ones((n_out - 1) * D + T, dtype=np.complex64)
    bad = 600
    x[bad] = np.inf
    taps = np.full(T, 0.01, dtype=np.float32)
    y = _host(ops.fir(_dev(taps), _dev(x), D, n_out))
    touched = np.array([(k * D <= bad < k * D + T) for k in range(n_out)])
    assert np.all(np.isfinite(y[~touched]))
    assert np.all(~np.isfinite(y[touched]))


# firDecFFKernel: real taps x real samples, even D >= 4, ceil(T / D) <= 32 (the C5 audio FIR)
DEC_FF = [
    # (T, D, nOut): C5's audio filter small and large (many-phase path), a ragged last tap row,
    # 2 taps per phase, D > T, 32 taps per phase, a short tail block
    (255, 20, 625), (255, 20, 100_003), (250, 20, 5000), (7, 6, 2049), (3, 16, 100), (127, 4, 70_000),
    (255, 8, 1)]


@pytest.mark.parametrize("T,D,n_out", DEC_FF)
def test_fir_ff_phase_pair_kernel(ops, orc, T, D, n_out):
    rng = np.random.default_rng(T * 7 + D * 131 + n_out)
    n_in = (n_out - 1) * D + T
    taps = orc.lowpass_taps(T, 0.4 / D).astype(np.float32)
    x = rng.standard_normal(n_in).astype(np.float32)
    y64, bound = orc.fir_f64(taps, x, D, n_out)
    y = _host(ops.fir(_dev(taps), _dev(x), D, n_out))
    _check_fir(y, y64, bound, (T, D, n_out))
    # a misaligned input takes the per-output kernel: same per-element bound (a single cancelling
    # output makes the relative L2 figure meaningless)
    xd = _dev(np.concatenate([np.zeros(1, np.float32), x]))
    y = _host(ops.fir(_dev(taps), xd[1:], D, n_out))
    _check_fir(y, y64, bound, (T, D, n_out, "misaligned"), l2=n_out > 100)


def test_fir_ff_phase_pair_inf_stays_local(ops):
    T, D, n_out = 250, 20, 3000  # last tap row half empty: no zero tap x inf product
    x = np.ones((n_out - 1) * D + T, dtype=np.float32)
    for bad in (600, 20 * 511 + 250, len(x) - 1):
        xb = x.copy()
        xb[bad] = np.inf
        y = _host(ops.fir(_dev(np.full(T, 0.01, np.float32)), _dev(xb), D, n_out))
        touched = np.array([(k * D <= bad < k * D + T) for k in range(n_out)])
        assert np.all(np.isfinite(y[~touched])), bad
        assert np.all(~np.isfinite(y[touched])), bad


def test_int8_to_float_all_codes_bit_exact(ops, orc, golden_dir):
    g = np.load(os.path.join(golden_dir, "int8_golden.npz"))
    codes = np.tile(g["codes"], 9)  # 2304 elements: vector path + tail
    out = _host(ops.int8_to_norm_float(_dev(codes)))
    assert out.tobytes() == np.tile(g["table"], 9).tobytes()
    for off in (1, 5, 15):  # misaligned input -> scalar path
        out = _host(ops.int8_to_norm_float(_dev(codes)[off:]))
        assert out.tobytes() == orc.int8_to_float(codes[off:]).tobytes()


def test_am_demod_bit_exact(ops, orc, golden_dir):
    g = np.load(os.path.join(golden_dir, "am_golden.npz"))
    z = g["z"]
    out = _host(ops.quad_am_demod(_dev(z)))
    assert out.tobytes() == orc.quad_am_demod(z).tobytes()
    out = _host(ops.quad_am_demod(_dev(z)[1:]))  # odd start: scalar path
    assert out.tobytes() == orc.quad_am_demod(z[1:]).tobytes()


@pytest.mark.parametrize("T,D", [(127, 1), (1023, 10), (255, 20), (5, 1)])
def test_fused_chains_match_unfused_bit_exact(ops, orc, T, D):
    """On the fp32 VALU path, int8 -> FIR -> AM in one kernel == gsdrInt8ToNormFloat ->
    gsdrFirFC -> gsdrQuadAmDemod bit for bit. (The int8 MFMA path is checked against the oracle
    in test_int8_mfma_path.)"""
    import torch
    rng = np.random.default_rng(T + D)
    n_out = 5000
    n_in = (n_out - 1) * D + T
    iq = rng.integers(-128, 128, size=2 * n_in).astype(np.int8)
    taps = orc.lowpass_taps(T, 0.2 / D if D > 1 else 0.1)
    iq_d, taps_d = _dev(iq), _dev(taps)
    prev = ops.set_kernel_policy(ops.POLICY_NO_MFMA)
    try:
        xf = ops.int8_to_norm_float(iq_d).view(torch.complex64)
        y_unfused = ops.fir(taps_d, xf, D, n_out)
        am_unfused = ops.quad_am_demod(y_unfused)
        y_fused = ops.fir(taps_d, iq_d, D, n_out, int8_iq=True)
        am_fused = ops.fir(taps_d, iq_d, D, n_out, int8_iq=True, am=True)
        am_fir_fused = ops.fir(taps_d, xf, D, n_out, am=True)
        assert _host(y_fused).tobytes() == _host(y_unfused).tobytes()
        assert _host(am_fused).tobytes() == _host(am_unfused).tobytes()
        assert _host(am_fir_fused).tobytes() == _host(am_unfused).tobytes()
    finally:
        ops.set_kernel_policy(prev)
    # and against the float64 oracle
    x = orc.int8_to_float(iq).view(np.complex64)
    y64, bound = orc.fir_f64(taps, x, D, n_out)
    assert np.all(np.abs(_host(am_fused) - np.abs(y64)) <= FIR_TOL * bound + 1e-30)


MFMA_CASES = [(1, 1), (2, 7), (31, 2048), (32, 2049), (33, 4095), (63, 777), (64, 65536), (65, 3),
              (96, 10000), (127, 50000), (128, 2047), (129, 123457)]


@pytest.mark.parametrize("T,n_out", MFMA_CASES)
def test_int8_mfma_path(ops, orc, T, n_out):
    """Exact int8 MFMA FIR (D = 1, T <= 129): against the float64 oracle, AM consistent with the
    complex output bit for bit, and against the fp32 VALU kernel within the tolerance."""
    import torch
    rng = np.random.default_rng(T * 7 + n_out)
    n_in = n_out - 1 + T
    iq = rng.integers(-128, 128, size=2 * n_in).astype(np.int8)
    iq[:64] = -128  # the clamp -128 -> -127 must be exact
    taps = (orc.lowpass_taps(T, 0.1) if T > 2 else rng.standard_normal(T)).astype(np.float32)
    taps[T // 2] *= -1.5
    iq_d, taps_d = _dev(iq), _dev(taps)
    y = _host(ops.fir(taps_d, iq_d, 1, n_out, int8_iq=True))
    am = _host(ops.fir(taps_d, iq_d, 1, n_out, int8_iq=True, am=True))
    x = orc.int8_to_float(iq).view(np.complex64)
    y64, bound = orc.fir_f64(taps, x, 1, n_out)
    _check_fir(y, y64, bound, ("mfma", T, n_out))
    # the MFMA epilogue forms |y| from the unscaled accumulators with the hardware square root
    # (v_sqrt_f32, <= 1 ulp) and scales once: a few ulp from AM of the rounded complex output
    am_ref = orc.quad_am_demod(y)
    assert np.all(np.abs(am - am_ref) <= 4 * np.spacing(am_ref))
    assert np.all(np.abs(am - np.abs(y64)) <= FIR_TOL * bound + 1e-30)
    prev = ops.set_kernel_policy(ops.POLICY_NO_MFMA)
    try:
        y_valu = _host(ops.fir(taps_d, iq_d, 1, n_out, int8_iq=True))
    finally:
        ops.set_kernel_policy(prev)
    assert np.all(np.abs(y.astype(np.complex128) - y_valu) <= 2 * FIR_TOL * bound + 1e-30)
    del torch


def test_int8_mfma_misaligned_falls_back(ops, orc):
    rng = np.random.default_rng(77)
    T, n_out = 127, 3000
    iq = rng.integers(-128, 128, size=2 * (n_out + T) + 16).astype(np.int8)
    taps = orc.lowpass_taps(T, 0.1)
    for off in (2, 4, 6, 14):  # every even misalignment class of the split pass
        y = _host(ops.fir(_dev(taps), _dev(iq)[off:], 1, n_out, int8_iq=True))
        y64, bound = orc.fir_f64(taps, orc.int8_to_float(iq[off:]).view(np.complex64), 1, n_out)
        _check_fir(y, y64, bound, ("misaligned", off))


I8_DEC_CASES = [(1023, 10, 20000), (1023, 10, 1), (255, 5, 3001), (64, 3, 777), (300, 1, 5000),
                (1346, 2, 2049), (127, 16, 4096), (1023, 2, 777)]


@pytest.mark.parametrize("T,D,n_out", I8_DEC_CASES)
def test_int8_decimating_mfma_path(ops, orc, T, D, n_out):
    """int8 IQ x real taps on the split-K Toeplitz f16 MFMA kernel (D > 1 or T > 129; the C5 RF
    stage): against the float64 oracle, AM within a few ulp of AM of the complex output, and
    against the fp32 VALU kernel."""
    rng = np.random.default_rng(T * 13 + D)
    n_in = (n_out - 1) * D + T
    iq = rng.integers(-128, 128, size=2 * n_in).astype(np.int8)
    iq[:64] = -128
    taps = orc.lowpass_taps(T, 0.4 / D).astype(np.float32)
    taps[T // 3] *= -2.0
    iq_d, taps_d = _dev(iq), _dev(taps)
    with _Policy(ops, ops.POLICY_NO_FFT):
        y = _host(ops.fir(taps_d, iq_d, D, n_out, int8_iq=True))
        am = _host(ops.fir(taps_d, iq_d, D, n_out, int8_iq=True, am=True))
    x = orc.int8_to_float(iq).view(np.complex64)
    y64, bound = orc.fir_f64(taps, x, D, n_out)
    _check_fir(y, y64, bound, ("i8-dec-mfma", T, D, n_out))
    am_ref = orc.quad_am_demod(y)
    assert np.all(np.abs(am - am_ref) <= 4 * np.spacing(am_ref))
    assert np.all(np.abs(am - np.abs(y64)) <= FIR_TOL * bound + 1e-30)
    prev = ops.set_kernel_policy(ops.POLICY_NO_MFMA)
    try:
        y_valu = _host(ops.fir(taps_d, iq_d, D, n_out, int8_iq=True))
    finally:
        ops.set_kernel_policy(prev)
    assert np.all(np.abs(y.astype(np.complex128) - y_valu) <= 2 * FIR_TOL * bound + 1e-30)


@pytest.mark.parametrize("T,D,n_out,off", [(1023, 10, 400_000, 0), (1023, 10, 130_001, 2), (255, 4, 200_000, 6),
                                           (1346, 2, 150_000, 0), (64, 3, 90_000, 4)])
def test_int8_decimating_wave_specialised_bit_exact(ops, orc, T, D, n_out, off):
    """The r01-r04 8-way wave-specialised int8 decimating kernel (GSDR_POLICY_I8_WS8: producer waves
    convert, 8 consumer waves split K) is bit-identical to the barrier-synchronous one, at several tiles
    per block and at 2-byte-misaligned inputs. The default 4-way kernel (r05: one consumer wave per SIMD,
    a quarter of K each) groups the K sums differently: it is within the float64 bound on a prefix, and
    within twice it of the synchronous kernel everywhere."""
    rng = np.random.default_rng(T + D + off)
    n_in = (n_out - 1) * D + T
    iq = rng.integers(-128, 128, size=2 * n_in + off).astype(np.int8)
    taps = orc.lowpass_taps(T, 0.4 / D).astype(np.float32)
    iq_d, taps_d = _dev(iq)[off:], _dev(taps)
    for am in (False, True):
        with _Policy(ops, ops.POLICY_NO_FFT | ops.POLICY_I8_WS8):
            y_ws8 = _host(ops.fir(taps_d, iq_d, D, n_out, int8_iq=True, am=am))
        with _Policy(ops, ops.POLICY_NO_WS | ops.POLICY_NO_FFT):
            y_sync = _host(ops.fir(taps_d, iq_d, D, n_out, int8_iq=True, am=am))
        assert y_ws8.tobytes() == y_sync.tobytes(), ("i8-ws8-vs-sync", T, D, n_out, off, am)
    m = min(n_out, 5000)
    x = orc.int8_to_float(iq[off: off + 2 * ((m - 1) * D + T)]).view(np.complex64)
    y64, bound = orc.fir_f64(taps, x, D, m)
    with _Policy(ops, ops.POLICY_NO_FFT):
        y_ws = _host(ops.fir(taps_d, iq_d, D, n_out, int8_iq=True))
    _check_fir(y_ws[:m], y64, bound, ("i8-ws4", T, D, off))
    with _Policy(ops, ops.POLICY_NO_FFT | ops.POLICY_I8_WS8):
        y_ws8 = _host(ops.fir(taps_d, iq_d, D, n_out, int8_iq=True))
    _check_fir(y_ws8[:m], y64, bound, ("i8-ws8", T, D, off))
    # everywhere: |y4 - y8| <= 2e-6 sum|h||x|, sum|h||x| <= sum|h| max|x| (max |x| = 1 after the convert)
    assert np.max(np.abs(y_ws - y_ws8)) <= 2 * FIR_TOL * np.abs(taps).sum() * 1.01, ("i8-ws4-vs-ws8", T, D)


def test_int8_decimating_mfma_misaligned(ops, orc):
    """Any sample-aligned input takes the MFMA kernel (dword loads + byte funnel shift)."""
    rng = np.random.default_rng(78)
    T, D, n_out = 1023, 10, 3000
    iq = rng.integers(-128, 128, size=2 * ((n_out - 1) * D + T) + 16).astype(np.int8)
    taps = orc.lowpass_taps(T, 0.04)
    for off in (2, 4, 6, 14):
        with _Policy(ops, ops.POLICY_NO_FFT):
            y = _host(ops.fir(_dev(taps), _dev(iq)[off:], D, n_out, int8_iq=True))
        y64, bound = orc.fir_f64(taps, orc.int8_to_float(iq[off:]).view(np.complex64), D, n_out)
        _check_fir(y, y64, bound, ("i8-dec-misaligned", off))


CF_MFMA_CASES = [(64, 1, 1000), (127, 3, 5000), (255, 2, 777), (1023, 10, 20000), (1023, 1, 4113),
                 (600, 16, 3000), (1023, 5, 1), (300, 7, 2049)]


@pytest.mark.parametrize("T,D,n_out", CF_MFMA_CASES)
def test_cf_mfma_path(ops, orc, T, D, n_out):
    """Split-precision bf16 MFMA FIR (cf32 x real taps, T >= 64): against the float64 oracle,
    the AM epilogue bit-identical to AM of the complex output, and against the fp32 VALU kernel."""
    rng = np.random.default_rng(T * 11 + D)
    n_in = (n_out - 1) * D + T
    x = (rng.standard_normal(n_in) + 1j * rng.standard_normal(n_in)).astype(np.complex64)
    taps = orc.lowpass_taps(T, 0.4 / D).astype(np.float32)
    x_d, taps_d = _dev(x), _dev(taps)
    with _Policy(ops, ops.POLICY_NO_FFT):
        y = _host(ops.fir(taps_d, x_d, D, n_out))
        am = _host(ops.fir(taps_d, x_d, D, n_out, am=True))
    y64, bound = orc.fir_f64(taps, x, D, n_out)
    _check_fir(y, y64, bound, ("cf-mfma", T, D, n_out))
    assert am.tobytes() == orc.quad_am_demod(y).tobytes()
    prev = ops.set_kernel_policy(ops.POLICY_NO_MFMA)
    try:
        y_valu = _host(ops.fir(taps_d, x_d, D, n_out))
    finally:
        ops.set_kernel_policy(prev)
    assert np.all(np.abs(y.astype(np.complex128) - y_valu) <= 2 * FIR_TOL * bound + 1e-30)


@pytest.mark.parametrize("no_fft", [True, False])
def test_cf_mfma_dynamic_range(ops, orc, no_fft):
    """Bursts 1e6 apart in amplitude inside one tile window: the MFMA kernels keep every output
    within 1e-6 of its OWN window's sum |h||x| (their per-tile direct path); with the FFT kernel
    (no_fft=False) the blocks straddling a burst edge take its direct-form fallback."""
    T, D, n_out = 1023, 10, 12000
    rng = np.random.default_rng(5)
    n_in = (n_out - 1) * D + T
    x = (rng.standard_normal(n_in) + 1j * rng.standard_normal(n_in)).astype(np.complex64)
    amp = np.where((np.arange(n_in) // 3000) % 2 == 0, 1.0, 1e-6).astype(np.float32)
    x = (x * amp).astype(np.complex64)
    taps = orc.lowpass_taps(T, 0.04).astype(np.float32)
    with _Policy(ops, ops.POLICY_NO_FFT if no_fft else 0):
        y = _host(ops.fir(_dev(taps), _dev(x), D, n_out))
    y64, bound = orc.fir_f64(taps, x, D, n_out)
    _check_fir(y, y64, bound, ("dynamic-range", no_fft))


@pytest.mark.parametrize("T,D,n_out,quiet", [(1023, 10, 300_000, True), (1023, 1, 200_000, False),
                                             (255, 4, 150_001, True), (64, 2, 70_000, False)])
def test_cf_mfma_wave_specialised_matches_sync(ops, orc, T, D, n_out, quiet):
    """The wave-specialised (producer / consumer) cf32 MFMA kernel performs the same arithmetic in
    the same order as the barrier-synchronous one, also across direct-path tiles (quiet
    stretches) and with several tiles per block; and stays within tolerance of float64."""
    rng = np.random.default_rng(T + 7 * D)
    n_in = (n_out - 1) * D + T
    x = (rng.standard_normal(n_in) + 1j * rng.standard_normal(n_in)).astype(np.complex64)
    if quiet:
        x[(np.arange(n_in) // 20_000) % 5 == 3] *= np.float32(1e-7)
    taps = orc.lowpass_taps(T, 0.4 / D).astype(np.float32)
    x_d, taps_d = _dev(x), _dev(taps)
    for am in (False, True):
        with _Policy(ops, ops.POLICY_NO_FFT):
            y_ws = _host(ops.fir(taps_d, x_d, D, n_out, am=am))
        with _Policy(ops, ops.POLICY_NO_WS | ops.POLICY_NO_FFT):
            y_sync = _host(ops.fir(taps_d, x_d, D, n_out, am=am))
        # identical arithmetic; only the K-padding units that the synchronous kernel also folds
        # into a tile's scale statistics may move a tile's scale (or direct decision)
        diff = y_ws != y_sync
        assert diff.mean() <= 0.01, ("ws-vs-sync", T, D, n_out, am, int(diff.sum()))
        assert np.max(np.abs(y_ws - y_sync)) <= 1e-6 * np.max(np.abs(y_sync)), ("ws-vs-sync", T, D, am)
    sl = slice(0, min(n_out, 20_000))
    y64, bound = orc.fir_f64(taps, x[: (sl.stop - 1) * D + T], D, sl.stop)
    with _Policy(ops, ops.POLICY_NO_FFT):
        y_ws = _host(ops.fir(taps_d, x_d, D, n_out))[sl]
    _check_fir(y_ws, y64, bound, ("ws", T, D))


def test_ws_abort_is_reported(ops, orc):
    """A wave-specialised launch whose producer / consumer hand-off waits give up is not silent:
    with the spin limit at 0 every wait that is not already satisfied aborts, the launch drains and
    counts it in the host-visible word (gsdrAmdWsAborts), and the next wave-specialised launch on
    the device reports hipErrorLaunchTimeOut instead of returning. After the report the count is
    clear and a normal launch is correct again."""
    from gpusdr._native import HipError
    T, D, n_out = 1023, 10, 100_000
    n_in = (n_out - 1) * D + T
    x = orc.synth_wideband_cf32(0xAB, 0.013, 0.31, 0, n_in)
    taps = orc.lowpass_taps(T, 0.04, "blackman")
    x_d, taps_d = _dev(x), _dev(taps)
    with _Policy(ops, ops.POLICY_NO_FFT):
        assert ops.fir_kernel_class(x_d, taps_d, D) == "cf-mfma"
        assert ops.ws_aborts(reset=True) == 0
        prev = ops.set_ws_spin_limit(0)
        try:
            ops.fir(taps_d, x_d, D, n_out)
            assert ops.ws_aborts(reset=False) > 0
        finally:
            ops.set_ws_spin_limit(prev)
        with pytest.raises(HipError, match="gsdrFirFC"):
            ops.fir(taps_d, x_d, D, n_out)
        assert ops.ws_aborts(reset=False) == 0
        y = _host(ops.fir(taps_d, x_d, D, n_out))
        assert ops.ws_aborts(reset=True) == 0
    y64, bound = orc.fir_f64(taps, x, D, n_out)
    _check_fir(y, y64, bound, "after-abort")


def test_cf_mfma_misaligned_falls_back(ops, orc):
    T, D, n_out = 255, 4, 3000
    rng = np.random.default_rng(9)
    n_in = (n_out - 1) * D + T
    x = (rng.standard_normal(n_in + 1) + 1j * rng.standard_normal(n_in + 1)).astype(np.complex64)
    taps = orc.lowpass_taps(T, 0.1).astype(np.float32)
    y = _host(ops.fir(_dev(taps), _dev(x)[1:], D, n_out))  # 8-byte aligned: the VALU kernel
    y64, bound = orc.fir_f64(taps, x[1:], D, n_out)
    _check_fir(y, y64, bound, "cf-misaligned")


@pytest.mark.parametrize("T,L,mfma", [(127, 10000, True), (127, 50, True), (33, 4099, True), (127, 10000, False),
                                       (1, 300, True)])
def test_fir_carry_streaming(ops, orc, T, L, mfma):
    """gsdrInt8FirFCAmDemodCarry over a stream pushed in blocks of L samples into one buffer
    [history | block]: the in-place history carry makes the concatenated outputs those of one
    FIR over the whole stream. L = 50 < T - 1 takes the overlapping (bounce) carry."""
    import torch
    rng = np.random.default_rng(T * 3 + L)
    nblk, H = 5, T - 1
    stream = rng.integers(-128, 128, size=2 * (H + nblk * L)).astype(np.int8)
    taps = (orc.lowpass_taps(T, 0.1) if T > 2 else np.ones(T)).astype(np.float32)
    taps_d = _dev(taps)
    buf = torch.zeros(2 * (H + L), dtype=torch.int8, device="cuda")
    buf[: 2 * H] = _dev(stream[: 2 * H])
    prev = ops.set_kernel_policy(0 if mfma else ops.POLICY_NO_MFMA)
    outs = []
    try:
        for b in range(nblk):
            buf[2 * H:] = _dev(stream[2 * (H + b * L): 2 * (H + (b + 1) * L)])
            out = torch.empty(L, dtype=torch.float32, device="cuda")
            ops.fir_am_i8_carry(taps_d, buf, 1, L, out, buf[: 2 * H])
            outs.append(_host(out))
    finally:
        ops.set_kernel_policy(prev)
    am = np.concatenate(outs)
    x = orc.int8_to_float(stream).view(np.complex64)
    y64, bound = orc.fir_f64(taps, x, 1, nblk * L)
    assert np.all(np.abs(am - np.abs(y64)) <= FIR_TOL * bound + 1e-30), (T, L, mfma)
    assert _host(buf[: 2 * H]).tobytes() == stream[len(stream) - 2 * H:].tobytes()


@pytest.mark.parametrize("T,D,n1,n2", [(1023, 10, 5000, 7000), (255, 4, 333, 1000), (64, 3, 100, 50)])
def test_fir_carry_decimating(ops, orc, T, D, n1, n2):
    """gsdrInt8FirFCAmDemodCarry with D > 1: the carry is the unconsumed tail of the call's input,
    samples [n1 D, (n1 - 1) D + T) (T - D of them). Put directly in front of the stream's next
    samples it makes two chained calls equal one call over the whole stream."""
    import torch
    rng = np.random.default_rng(T + D)
    n_in1 = (n1 - 1) * D + T
    n_all = (n1 + n2 - 1) * D + T
    stream = rng.integers(-128, 128, size=2 * n_all).astype(np.int8)
    taps_d = _dev(orc.lowpass_taps(T, 0.4 / D).astype(np.float32))
    out1 = torch.empty(n1, dtype=torch.float32, device="cuda")
    buf = torch.zeros(2 * (n_all - n1 * D), dtype=torch.int8, device="cuda")  # [carry | rest]
    ops.fir_am_i8_carry(taps_d, _dev(stream[: 2 * n_in1]), D, n1, out1, buf[: 2 * (T - D)])
    buf[2 * (T - D):] = _dev(stream[2 * n_in1:])
    # the reference count rule floor((N - (T - 1)) / D) (Fir.cpp:178-186) yields n2 - 1 here for D > 1
    n2 = ops.fir_output_count(buf.numel() // 2, T, D)
    out2 = torch.empty(n2, dtype=torch.float32, device="cuda")
    ops.fir_am_i8_carry(taps_d, buf, D, n2, out2, torch.empty(2 * (T - D), dtype=torch.int8, device="cuda"))
    chained = np.concatenate([_host(out1), _host(out2)])
    x = orc.int8_to_float(stream).view(np.complex64)
    y64, bound = orc.fir_f64(_host(taps_d), x, D, n1 + n2)  # one FIR over the whole stream
    assert np.all(np.abs(chained - np.abs(y64)) <= FIR_TOL * bound + 1e-30), (T, D)


def test_cosine_sources(ops, orc):
    # CosineSourceTests.cpp:8-56 KAT plus the oracle over a longer run
    delta = np.float32(2.0 * np.pi * 1.0 / 100.0)
    z = _host(ops.cosine(0.0, float(np.float32(104) * delta), 104, True))
    theta = np.arange(101, dtype=np.float32) * np.float32(0.01) * np.float32(np.pi) * np.float32(2)
    assert np.all(np.abs(z[:101].real - np.cos(theta)) < 1e-4)
    assert np.all(np.abs(z[:101].imag - np.sin(theta)) < 1e-4)
    f = _host(ops.cosine(0.25, 1000.25, 1 << 16, False))
    assert np.max(np.abs(f - orc.cosine_f(0.25, 1000.25, 1 << 16))) < 2e-5


def test_synth_sources_match_oracle(ops, orc):
    n = 100_000
    a = _host(ops.synth_iq_int8(0x5EED, 20e6, 1e3, 1.5e6, 12345, n))
    b = orc.synth_iq_int8(0x5EED, 20e6, 1e3, 1.5e6, 12345, n)
    diff = np.abs(a.astype(np.int32) - b.astype(np.int32))
    assert diff.max() <= 1 and np.mean(diff == 0) > 0.999
    w = _host(ops.synth_wideband_cf32(0xC3, 0.013, 0.31, 777, n))
    assert np.max(np.abs(w - orc.synth_wideband_cf32(0xC3, 0.013, 0.31, 777, n))) < 1e-5


def test_large_chain_sampled_parity(ops, orc):
    """C3-sized stream (2^24 cf32, 1023 taps, D=10): spot-check 2000 outputs against float64."""
    import torch
    n_in = 1 << 24
    T, D = 1023, 10
    taps = orc.lowpass_taps(T, 0.04, "blackman")
    x = ops.synth_wideband_cf32(0xC3, 0.013, 0.31, 0, n_in)
    n_out = ops.fir_output_count(n_in, T, D)
    am = ops.fir(_dev(taps), x, D, n_out, am=True)
    rng = np.random.default_rng(5)
    ks = np.sort(rng.choice(n_out, 2000, replace=False))
    ks[-1] = n_out - 1
    ks[0] = 0
    xh = _host(x)
    amh = _host(am)
    for k in ks:
        seg = xh[k * D: k * D + T]
        y64, bound = orc.fir_f64(taps, seg, D, 1)
        assert abs(amh[k] - abs(y64[0])) <= FIR_TOL * bound[0], int(k)
    del torch


def test_graph_capture_replay(ops, orc):
    """The steady-state chain step is capturable into a HIP graph and replays correctly."""
    import torch
    T, D, n_out = 127, 1, 1 << 16
    n_in = n_out - 1 + T
    taps = _dev(orc.lowpass_taps(T, 0.1))
    iq = ops.synth_iq_int8(7, 20e6, 1e3, 1.5e6, 0, n_in)
    out = torch.empty(n_out, device="cuda")
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        ops.fir(taps, iq, D, n_out, out=out, int8_iq=True, am=True)  # warm-up (sets LDS attrs)
    torch.cuda.current_stream().wait_stream(s)
    ref = _host(out).copy()
    g = torch.cuda.CUDAGraph()
    out.zero_()
    with torch.cuda.graph(g):
        ops.fir(taps, iq, D, n_out, out=out, int8_iq=True, am=True)
    g.replay()
    assert _host(out).tobytes() == ref.tobytes()
    ops.synth_iq_int8(8, 20e6, 1e3, 1.5e6, 0, n_in, out=iq)  # new data, same buffers
    g.replay()
    x = orc.int8_to_float(_host(iq)).view(np.complex64)
    y64, bound = orc.fir_f64(_host(taps), x, D, n_out)
    assert np.all(np.abs(_host(out) - np.abs(y64)) <= FIR_TOL * bound)


def test_multiply_cc_bit_exact(ops, orc):
    rng = np.random.default_rng(31)
    for n in (1, 7, 4096, 100003):
        a = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
        b = (rng.standard_normal(n) * 1e3 + 1j * rng.standard_normal(n)).astype(np.complex64)
        got = _host(ops.multiply_cc(_dev(a), _dev(b)))
        assert got.tobytes() == orc.multiply_cc(a, b).tobytes()


def test_quad_fm_demod_kernel(ops, orc):
    rng = np.random.default_rng(32)
    gain = orc.fm_gain(2.4e5, 7.5e4)
    for n in (2, 3, 1000, 65537):
        z = ((rng.standard_normal(n) + 1j * rng.standard_normal(n)) * 10.0 ** rng.uniform(-3, 3, n)).astype(np.complex64)
        got = _host(ops.quad_fm_demod(_dev(z), gain))
        want = orc.quad_fm_demod_f64(z, gain)
        assert len(got) == n - 1
        assert np.all(np.abs(got - want) <= abs(gain) * 4 * np.spacing(np.float32(np.pi)) +
                      2 * np.spacing(np.abs(want).astype(np.float32)))


@pytest.mark.parametrize("kind,T,D,n_out", [("c64", 127, 1, 5000), ("c64", 1023, 10, 3000), ("i8", 127, 1, 70000),
                                             ("i8", 1023, 10, 20000), ("c64", 64, 3, 1), ("i8", 255, 4, 777),
                                             # FFT kernel shapes (T >= 256, D in 2..10): the row chirp /
                                             # c_p-in-G / per-block factor decomposition
                                             ("c64", 1023, 10, 200_000), ("c64", 1023, 4, 60_000),
                                             ("c64", 300, 2, 50_001), ("i8", 1023, 10, 150_000),
                                             ("i8", 511, 6, 40_000)])
def test_fused_frequency_shift_fir(ops, orc, kind, T, D, n_out):
    """Frequency shifter fused into the FIR load (gsdr*MixFirFC*): against the oracle mixer
    (exact 64-bit phase, float32 angle, float64 exponential) and float64 FIR; the AM variant
    against |y|; and streaming: two calls with phase0 advanced by the consumed samples equal one."""
    rng = np.random.default_rng(T + D + n_out)
    n_in = (n_out - 1) * D + T
    phase0, step = 1.2345, -2 * np.pi * 0.15
    taps = orc.lowpass_taps(T, 0.4 / D)
    if kind == "c64":
        x = (rng.standard_normal(n_in) + 1j * rng.standard_normal(n_in)).astype(np.complex64)
        xd, xf = _dev(x), x
    else:
        iq = rng.integers(-128, 128, size=2 * n_in).astype(np.int8)
        xd, xf = _dev(iq), orc.int8_to_float(iq).view(np.complex64)
    td = _dev(taps)
    y = _host(ops.fir(td, xd, D, n_out, int8_iq=(kind == "i8"), mix=(phase0, step)))
    am = _host(ops.fir(td, xd, D, n_out, int8_iq=(kind == "i8"), am=True, mix=(phase0, step)))
    mixed = orc.mix_f64(xf, phase0, step)
    y64, bound = orc.fir_f64(taps, mixed.astype(np.complex64), D, n_out)
    _check_fir(y, y64, bound, ("mix", kind, T, D))
    assert np.all(np.abs(am - np.abs(y64)) <= FIR_TOL * bound + 1e-30)
    if n_out >= 4:
        h = n_out // 2
        w = 2 if kind == "i8" else 1
        y1 = _host(ops.fir(td, xd, D, h, int8_iq=(kind == "i8"), mix=(phase0, step)))
        y2 = _host(ops.fir(td, xd[w * h * D:], D, n_out - h, int8_iq=(kind == "i8"),
                           mix=(np.fmod(phase0 + h * D * step, 2 * np.pi), step)))
        _check_fir(np.concatenate([y1, y2]), y64, bound, ("mix-stream", kind, T, D))


@pytest.mark.parametrize("kind,T,D,n_out", [("c64", 127, 4, 300_000), ("c64", 1023, 10, 30_000), ("i8", 255, 8, 40_000),
                                             ("c64", 20000, 10, 300)])
def test_fused_fm_front(ops, orc, kind, T, D, n_out):
    """Mixer -> low-pass, decimate -> FM discriminator in ONE kernel (gsdr*MixFirFCFmDemod): bit-exact
    against gsdrMixFirFC followed by gsdrQuadFmDemod where both run the LDS kernel (the first case,
    enough tiles; the direct-kernel case too), and within the FIR tolerance carried through the
    discriminator against the float64 oracle: |d arg| <= |dy_k|/|y_k| + |dy_k+1|/|y_k+1|."""
    rng = np.random.default_rng(T * 7 + D)
    n_in = n_out * D + T
    phase0, step = 0.4, 2 * np.pi * 0.03
    gain = orc.fm_gain(48000.0, 5000.0)
    taps = orc.lowpass_taps(T, 0.3 / D)
    if kind == "c64":
        i = np.arange(n_in)
        x = (np.exp(1j * (-step * i + 3.0 * np.sin(2 * np.pi * 1e-4 * i)))
             + 0.05 * (rng.standard_normal(n_in) + 1j * rng.standard_normal(n_in))).astype(np.complex64)
        xd, xf = _dev(x), x
    else:
        iq = rng.integers(-128, 128, size=2 * n_in).astype(np.int8)
        xd, xf = _dev(iq), orc.int8_to_float(iq).view(np.complex64)
    td = _dev(taps)
    fm = _host(ops.fm_front(td, xd, D, n_out, phase0, step, gain, int8_iq=(kind == "i8")))
    y = ops.fir(td, xd, D, n_out + 1, int8_iq=(kind == "i8"), mix=(phase0, step))
    unfused = _host(ops.quad_fm_demod(y, gain))
    if kind == "c64" and (n_out >= 100_000 or T > 10_000):
        assert fm.tobytes() == unfused.tobytes()
    mixed = orc.mix_f64(xf, phase0, step)
    y64, bound = orc.fir_f64(taps, mixed.astype(np.complex64), D, n_out + 1)
    want = gain * np.angle(y64[1:] * np.conj(y64[:-1]))
    rel = FIR_TOL * bound / np.maximum(np.abs(y64), 1e-30)
    tol = abs(gain) * (rel[:-1] + rel[1:] + 4e-7) + 1e-30
    d = np.abs(fm - want)
    d = np.minimum(d, np.abs(d - 2 * np.pi * abs(gain)))  # a branch-cut flip of arg near +-pi
    assert np.all(d <= tol), (kind, T, D, float(np.max(d / tol)))


def test_fm_demod_reference_entry(ops, orc):
    """gsdrFmDemod, the reference's call (fm_simpletest.cpp:400-413): stream offset, channel shift
    and QuadDemodFactory gain at the discriminator's rate, equal to the generic fused entry."""
    rf_rate, tuned, channel, dev_hz, D, first = 4_800_000, 97.5e6, 98.5e6, 75e3, 10, 123_456
    T, n_out = 255, 20_000
    taps = orc.lowpass_taps(T, 0.04)
    rng = np.random.default_rng(3)
    x = (rng.standard_normal(n_out * D + T) + 1j * rng.standard_normal(n_out * D + T)).astype(np.complex64)
    xd, td = _dev(x), _dev(taps)
    got = _host(ops.fm_demod(rf_rate, tuned, channel, dev_hz, D, first, td, xd, n_out))
    f32 = np.float32
    step = 2 * np.pi * (float(f32(tuned)) - float(f32(channel))) / rf_rate
    gain = float(f32(f32(rf_rate) / f32(D)) / (f32(2.0) * f32(np.pi) * f32(dev_hz) * f32(5)))
    ref = _host(ops.fm_front(td, xd, D, n_out, step * first, step, gain))
    assert got.tobytes() == ref.tobytes()


def test_zero_length_calls_are_no_ops(ops):
    """Every entry point called with 0 outputs / elements (an empty chunk, as a SteppingDriver step
    with nothing buffered produces) succeeds, launches nothing and writes nothing - through the
    C ABI directly, null data pointers included (Fir.cpp:221-223 returns before the kernel when
    nOut is 0)."""
    import ctypes

    import torch
    from gpusdr._native import lib
    L = lib()
    sentinel = torch.full((64,), 7.0, dtype=torch.float32, device="cuda")
    x = torch.zeros(64, dtype=torch.complex64, device="cuda")
    taps = torch.ones(8, dtype=torch.float32, device="cuda")
    stream = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    calls = []
    for name in sorted(set(ops._FIR_ENTRY.values())):
        calls.append((name, lambda f, o: f(1, taps.data_ptr(), 8, x.data_ptr(), o, 0, 0, stream)))
        calls.append((name + "(null)", lambda f, o: f(1, None, 8, None, None, 0, 0, stream)))
    for name in sorted(set(ops._MIX_ENTRY.values())):
        calls.append((name, lambda f, o: f(2, taps.data_ptr(), 8, x.data_ptr(), ctypes.c_double(0.0),
                                           ctypes.c_double(0.1), o, 0, 0, stream)))
    torch.cuda.synchronize()
    for name, call in calls:
        fn = getattr(L, name.split("(")[0])
        assert call(fn, sentinel.data_ptr()) == 0, name
    assert L.gsdrQuadAmDemod(x.data_ptr(), sentinel.data_ptr(), 0, 0, stream) == 0
    assert L.gsdrInt8ToNormFloat(None, None, 0, 0, stream) == 0
    assert L.gsdrMultiplyCC(None, None, None, 0, 0, stream) == 0
    assert L.gsdrQuadFmDemod(None, None, ctypes.c_float(1.0), 0, 0, stream) == 0
    assert L.gsdrCosineF(ctypes.c_float(0.0), ctypes.c_float(1.0), None, 0, 0, stream) == 0
    torch.cuda.synchronize()
    assert torch.all(sentinel == 7.0)


@pytest.mark.parametrize("kind", ["c64", "i8"])
def test_mixed_long_filter_runs_on_fft_kernel(ops, orc, kind):
    """A mixed long filter (gsdrMixFirFC*, 1023 taps, D = 10) takes the FFT kernel (it
    fell back to the VALU direct form): with the accuracy guard forced to 0 every FFT block goes to
    the kernel's direct-form fallback, which the block counter shows; that fallback (per-sample
    rotation) and the FFT path (decomposed rotation) both meet the float64 oracle, AM and complex."""
    T, D, n_out = 1023, 10, 60_000
    n_in = (n_out - 1) * D + T
    rng = np.random.default_rng(77)
    phase0, step = -0.7, 2 * np.pi * 0.0123
    taps = orc.lowpass_taps(T, 0.04)
    if kind == "c64":
        x = (rng.standard_normal(n_in) + 1j * rng.standard_normal(n_in)).astype(np.complex64)
        xd, xf = _dev(x), x
    else:
        iq = rng.integers(-128, 128, size=2 * n_in).astype(np.int8)
        xd, xf = _dev(iq), orc.int8_to_float(iq).view(np.complex64)
    td = _dev(taps)
    y64, bound = orc.fir_f64(taps, orc.mix_f64(xf, phase0, step).astype(np.complex64), D, n_out)
    ops.fft_direct_blocks(reset=True)
    prev = ops.set_fft_guard(0.0)
    try:
        y_dir = _host(ops.fir(td, xd, D, n_out, int8_iq=(kind == "i8"), mix=(phase0, step)))
        am_dir = _host(ops.fir(td, xd, D, n_out, int8_iq=(kind == "i8"), am=True, mix=(phase0, step)))
        assert ops.fft_direct_blocks(reset=True) > 0  # the FFT kernel ran (all its blocks direct)
    finally:
        ops.set_fft_guard(prev)
    y = _host(ops.fir(td, xd, D, n_out, int8_iq=(kind == "i8"), mix=(phase0, step)))
    am = _host(ops.fir(td, xd, D, n_out, int8_iq=(kind == "i8"), am=True, mix=(phase0, step)))
    assert ops.fft_direct_blocks(reset=True) == 0
    for yy, aa, what in ((y, am, "fft"), (y_dir, am_dir, "direct")):
        _check_fir(yy, y64, bound, ("mixed", kind, what))
        assert np.all(np.abs(aa - np.abs(y64)) <= FIR_TOL * bound + 1e-30), what


@pytest.mark.gpu
@pytest.mark.parametrize("i8", [False, True])
def test_bound_fir_launch_matches_fir(orc, i8):
    """ops.bind_fir (the bench's pre-validated launch) enqueues exactly ops.fir's kernel: bit-equal
    outputs, and it rejects an input too short for the outputs at bind time."""
    import torch
    from gpusdr import ops
    dev = torch.device("cuda", 0)
    T, D, n = 127, 1 if i8 else 10, 5000
    taps = torch.from_numpy(orc.lowpass_taps(T, 0.1)).to(dev)
    n_in = (n - 1) * D + T
    if i8:
        x = torch.randint(-128, 128, (2 * n_in,), dtype=torch.int8, device=dev)
    else:
        x = torch.randn(n_in, dtype=torch.complex64, device=dev)
    a = torch.empty(n, dtype=torch.float32, device=dev)
    b = torch.empty(n, dtype=torch.float32, device=dev)
    ops.fir(taps, x, D, n, out=a, am=True, int8_iq=i8)
    ops.bind_fir(taps, x, D, n, b, am=True, int8_iq=i8)()
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    with pytest.raises(ValueError):
        ops.bind_fir(taps, x[: x.numel() // 2], D, n, b, am=True, int8_iq=i8)
