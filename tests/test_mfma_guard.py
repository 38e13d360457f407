"""The matrix-core FIR kernels on adversarial inputs (r06).

The MFMA kernels multiply f16 limbs: the taps as two limbs under one block scale (hi + lo, each tap kept to
2^-22 of itself only while it lies within ~2^-17 of the largest tap), the cf32 samples as two limbs under a
per-tile scale. A window whose non-zero samples all sit under taps below that range - a Blackman filter's
tails at a zero-padded stream start, after an exact-zero gap, between sparse impulses - loses its output,
which the 1e-6 sum|h||x| bound does not allow. Each kernel therefore computes such tiles in
the direct fp32 form: the cf32 kernels send a tile with an exact-zero 64-sample block to their direct path
(the guard already sent quiet blocks there), the int8 kernels a tile whose window holds an exact-zero run.
Here: the FFT kernel's adversarial signals (tests/test_fft_fir.py) on the cf32 MFMA kernel, and zero-padded
starts and exact-zero gaps on the int8 kernels of C2 (127 taps, D = 1) and C5 (1023 taps, D = 10, plain and
the fused chain), against float64 per element. Reference arithmetic: Fir.cpp:229-269 (gsdrFirFC)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

FIR_TOL = 1e-6


@pytest.fixture(scope="module")
def ops():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gpusdr import ops
    return ops


def _dev(a):
    import torch
    return torch.from_numpy(np.ascontiguousarray(a)).cuda()


def _host(t):
    import torch
    torch.cuda.synchronize()
    return t.cpu().numpy()


class _Policy:
    def __init__(self, ops, flags):
        self.ops, self.flags = ops, flags

    def __enter__(self):
        self.prev = self.ops.set_kernel_policy(self.flags)

    def __exit__(self, *exc):
        self.ops.set_kernel_policy(self.prev)


def _check(y, y64, bound, what, tile_out=512):
    err = np.abs(y.astype(np.complex128) - y64)
    bad = np.nonzero(~(err <= FIR_TOL * bound + 1e-30))[0]
    assert bad.size == 0, (what, int(bad.size), [(int(k), int(k // tile_out), float(err[k] / (bound[k] + 1e-300)))
                                                 for k in bad[:8]])


def _adversarial(name, n, rng):
    x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
    i = np.arange(n)
    if name == "silence":
        x[(i // 7000) % 3 == 1] = 0
    elif name == "impulses":
        x = np.zeros(n, np.complex64)
        x[::997] = 1 + 1j
    elif name == "zero-start":
        x[: 5000] = 0
    return x


@pytest.mark.parametrize("name", ["silence", "impulses", "zero-start"])
@pytest.mark.parametrize("T,D,window", [(1023, 10, "blackman"), (200, 3, "blackman")])
def test_cf_mfma_adversarial(ops, orc, name, T, D, window):
    """cf32 x real taps on the wave-specialised f16 MFMA kernel (T = 200, D = 3 takes it by default: the
    FFT kernel needs D in {1, 2, 4, 6, 8, 10}; C3's shape under GSDR_POLICY_NO_FFT)."""
    n_out = 40_000
    n_in = (n_out - 1) * D + T
    x = _adversarial(name, n_in, np.random.default_rng(11))
    taps = orc.lowpass_taps(T, 0.4 / D, window)
    x_d, taps_d = _dev(x), _dev(taps)
    with _Policy(ops, ops.POLICY_NO_FFT):
        assert ops.fir_kernel_class(x_d, taps_d, D) == "cf-mfma"
        y = _host(ops.fir(taps_d, x_d, D, n_out))
        am = _host(ops.fir(taps_d, x_d, D, n_out, am=True))
    y64, bound = orc.fir_f64(taps, x, D, n_out)
    _check(y, y64, bound, ("cf-mfma", name, T, D))
    _check(am, np.abs(y64), bound, ("cf-mfma-am", name, T, D))


def test_cf_mfma_nonfinite_stays_local(ops, orc):
    """An inf / NaN sample reaches only the outputs whose window holds it, on the cf32 MFMA kernel."""
    T, D, n_out = 1023, 10, 20000
    n_in = (n_out - 1) * D + T
    x = orc.synth_wideband_cf32(7, 0.013, 0.31, 0, n_in)
    x[50_000] = np.inf
    x[120_003] = np.nan
    taps = orc.lowpass_taps(T, 0.04, "blackman")
    with _Policy(ops, ops.POLICY_NO_FFT):
        y = _host(ops.fir(_dev(taps), _dev(x), D, n_out))
    k = np.arange(n_out)
    touched = np.zeros(n_out, bool)
    for pos in (50_000, 120_003):
        touched |= (k * D <= pos) & (pos < k * D + T)
    leaked = np.nonzero(~np.isfinite(y) & ~touched)[0]
    assert leaked.size == 0, (int(leaked.size), leaked[:8].tolist(), (leaked[:8] // 512).tolist())
    y64, bound = orc.fir_f64(taps, x, D, n_out)
    _check(y[~touched], y64[~touched], bound[~touched], "nonfinite")


def _zero_gapped_iq(T, seed, n_sig=60_000):
    """int8 IQ: T + 500 zero samples, a signal, a zero gap of 2 T samples, the signal again, a short gap."""
    from oracle import synth_iq_int8
    sig = synth_iq_int8(0x5EED + seed, 1e9, 1e3, 7.5e7, 0, n_sig)
    half = 2 * (n_sig // 2)
    return np.concatenate([np.zeros(2 * (T + 500), np.int8), sig[:half], np.zeros(4 * T, np.int8), sig[half:],
                           np.zeros(2 * 37, np.int8)])


@pytest.mark.parametrize("T,D,cut,window,kernel", [(1023, 10, 0.04, "blackman", "i8-dec-mfma"),
                                                   (255, 5, 0.08, "blackman", "i8-dec-mfma"),
                                                   (127, 1, 0.1, "hamming", "i8-mfma")])
def test_int8_mfma_zero_padded_windows(ops, orc, T, D, cut, window, kernel):
    """C5's RF filter and C2's filter on the int8 MFMA kernels, over a stream with a zero-padded start and
    exact-zero gaps: AM and complex outputs against float64 per element."""
    iq = _zero_gapped_iq(T, T)
    n_in = len(iq) // 2
    n_out = (n_in - T) // D + 1
    taps = orc.lowpass_taps(T, cut, window)
    x_d, taps_d = _dev(iq), _dev(taps)
    assert ops.fir_kernel_class(x_d, taps_d, D, int8_iq=True) == kernel
    y = _host(ops.fir(taps_d, x_d, D, n_out, int8_iq=True))
    am = _host(ops.fir(taps_d, x_d, D, n_out, int8_iq=True, am=True))
    xc = orc.int8_to_float(iq).view(np.complex64)
    y64, bound = orc.fir_f64(taps, xc, D, n_out)
    _check(y, y64, bound, ("int8", kernel, T, D))
    _check(am, np.abs(y64), bound, ("int8-am", kernel, T, D))


def _burst_onset_iq(n, quiet, seed):
    """int8 IQ: +-quiet LSB of noise for the first half, then full-scale noise (a burst onset)."""
    rng = np.random.default_rng(seed)
    q = np.where(np.arange(2 * n) < n, rng.integers(-quiet, quiet + 1, 2 * n), rng.integers(-128, 128, 2 * n))
    return q.astype(np.int8)


@pytest.mark.parametrize("T,D,cut,window,kernel", [(1023, 10, 0.04, "blackman", "i8-dec-mfma"),
                                                   (255, 5, 0.08, "blackman", "i8-dec-mfma"),
                                                   (127, 1, 0.1, "hamming", "i8-mfma")])
def test_int8_mfma_burst_onset(ops, orc, T, D, cut, window, kernel):
    """VERDICT r05 item 3's int8 x int8 form fails here (tools/exp/q8_tap_error.py --burst: 1.7-2.4x the
    bound): the windows with a full-scale burst under the tail taps and +-1 LSB under the large ones. The
    product's f16 x 2 tap limbs keep each tap to 2^-22 of itself: per element within the bound."""
    iq = _burst_onset_iq(120_000, 1, T)
    n_in = len(iq) // 2
    n_out = (n_in - T) // D + 1
    taps = orc.lowpass_taps(T, cut, window)
    x_d, taps_d = _dev(iq), _dev(taps)
    assert ops.fir_kernel_class(x_d, taps_d, D, int8_iq=True) == kernel
    y = _host(ops.fir(taps_d, x_d, D, n_out, int8_iq=True))
    am = _host(ops.fir(taps_d, x_d, D, n_out, int8_iq=True, am=True))
    xc = orc.int8_to_float(iq).view(np.complex64)
    y64, bound = orc.fir_f64(taps, xc, D, n_out)
    _check(y, y64, bound, ("int8-burst", kernel, T, D))
    _check(am, np.abs(y64), bound, ("int8-burst-am", kernel, T, D))


def test_fused_chain_zero_padded_windows(ops, orc):
    """The fused C5 chain (RF FIR -> AM -> audio FIR in one launch) over the zero-gapped stream: the AM
    samples against float64 per element, the audio within the carried bound."""
    import torch
    T, D, Ta, Da = 1023, 10, 255, 20
    iq = _zero_gapped_iq(T, 3, n_sig=400_000)
    n_in = len(iq) // 2
    n_rf = (n_in - T) // D + 1
    n_audio = (n_rf - Ta) // Da + 1
    rf, au = orc.lowpass_taps(T, 0.04, "blackman"), orc.lowpass_taps(Ta, 0.02)
    am = torch.zeros(n_rf, dtype=torch.float32, device="cuda")
    audio = torch.empty(n_audio, dtype=torch.float32, device="cuda")
    ops.am_chain_fused(_dev(rf), _dev(iq), D, n_rf, am, 0, _dev(au), Da, n_audio, audio, store_am=True)
    xc = orc.int8_to_float(iq).view(np.complex64)
    y64, rf_bound = orc.fir_f64(rf, xc, D, n_rf)
    _check(_host(am), np.abs(y64), rf_bound, "fused-am")
    a64 = np.abs(y64)
    want, audio_bound = orc.fir_f64(au, a64.astype(np.float32), Da, n_audio)
    carried, _ = orc.fir_f64(np.abs(au), (FIR_TOL * (rf_bound + a64)).astype(np.float32), Da, n_audio)
    got = _host(audio)
    bad = np.nonzero(~(np.abs(got - want) <= carried + FIR_TOL * audio_bound + 1e-30))[0]
    assert bad.size == 0, (int(bad.size), bad[:8].tolist())
