"""The oracle against the reference's own known-answer tests and the numpy golden fixtures.

This pins oracle/liborcl.so before any GPU comparison trusts it (tests/golden/MANIFEST.json
lists the fixtures and their generator, oracle/make_golden.py)."""
import hashlib
import json
import os

import numpy as np
import pytest


def _load_json(golden_dir, name):
    with open(os.path.join(golden_dir, name)) as f:
        return json.load(f)


def test_manifest_hashes(golden_dir):
    manifest = _load_json(golden_dir, "MANIFEST.json")
    for name, digest in manifest.items():
        if name.startswith("_"):
            continue
        with open(os.path.join(golden_dir, name), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == digest, name


def _replay_kat(orc, kat):
    taps = np.array(kat["taps"], dtype=np.float32)
    model = orc.FirStreamModel(taps, kat["decimation"])
    for push in kat["pushes"]:
        model.push(np.array([complex(a, b) for a, b in push], dtype=np.complex64))
    outs = []
    for rd in kat["reads"]:
        cap = rd["capacity_elements"]
        if isinstance(cap, str):  # "2x getOutputDataSize": oversized buffer
            cap = 2 * model.output_count()
        y, _ = model.read(cap)
        outs.append((y, np.array([complex(a, b) for a, b in rd["expected"]])))
    return outs


@pytest.mark.parametrize("name", ["kat_fir_two_commits.json", "kat_fir_partial_reads.json"])
def test_fir_kats(orc, golden_dir, name):
    kat = _load_json(golden_dir, name)
    for y, expected in _replay_kat(orc, kat):
        assert y.shape == expected.shape
        assert np.all(np.abs(y.real - expected.real) < kat["abs_tol"])
        assert np.all(np.abs(y.imag - expected.imag) < kat["abs_tol"])


def test_fir_convolution_orientation_fails_kat(orc, golden_dir):
    """The KAT distinguishes correlation from convolution."""
    kat = _load_json(golden_dir, "kat_fir_two_commits.json")
    x = np.array([complex(a, b) for p in kat["pushes"] for a, b in p], dtype=np.complex64)
    y_conv, _ = orc.fir_f64(np.array(kat["taps"][::-1], dtype=np.float32), x, 2)
    expected = np.array([complex(a, b) for a, b in kat["reads"][0]["expected"]])
    assert np.max(np.abs(y_conv - expected)) > 0.05


def test_cosine_kat(orc, golden_dir):
    kat = _load_json(golden_dir, "kat_cosine_source.json")
    fs, f = kat["sampleRate"], kat["frequency"]
    delta = np.float32(2.0 * np.pi * f / fs)  # ComplexCosineSource.cpp:49-51 (double, then float)
    n = kat["buffer_elements"]
    phi_end = np.float32(0.0) + np.float32(n) * delta
    z = orc.cosine_c(0.0, float(phi_end), n)
    i = np.arange(kat["checked_elements"])
    theta = (i.astype(np.float32) * np.float32(f) / np.float32(fs) * np.float32(np.pi) * np.float32(2.0))
    assert np.all(np.abs(z[: len(i)].real - np.cos(theta)) < kat["abs_tol"])
    assert np.all(np.abs(z[: len(i)].imag - np.sin(theta)) < kat["abs_tol"])


def test_fir_count_rule_matches_reference_comments(orc):
    # Fir.cpp:142-176 worked examples: (taps, decimation) -> inputs needed for 1, 2, 3 outputs
    for (T, D), needs in {(7, 2): (8, 10, 12), (5, 3): (7, 10, 13)}.items():
        for k, n in enumerate(needs, start=1):
            assert orc.fir_output_count(n, T, D) == k
            assert orc.fir_output_count(n - 1, T, D) == k - 1
    # the size_t wrap cases of the reference are guarded, not reproduced
    assert orc.fir_output_count(3, 5, 3) == 0
    assert orc.fir_output_count(10, 2, 4) == 2  # floor((10 - 1) / 4)
    assert orc.fir_output_count(10, 0, 1) == 0


def test_fir_golden(orc, golden_dir):
    g = np.load(os.path.join(golden_dir, "fir_golden.npz"))
    keys = sorted({k.rsplit("_", 1)[0] for k in g.files})
    assert len(keys) == 36
    for key in keys:
        D = int(key.split("_D")[1])
        taps, x, y_ref, b_ref = g[key + "_taps"], g[key + "_x"], g[key + "_y"], g[key + "_bound"]
        y, b = orc.fir_f64(taps, x, D, len(y_ref))
        assert np.allclose(b, b_ref, rtol=1e-12, atol=0), key
        assert np.all(np.abs(y - y_ref) <= 1e-12 * b_ref + 1e-300), key


def test_int8_table_bit_exact(orc, golden_dir):
    g = np.load(os.path.join(golden_dir, "int8_golden.npz"))
    out = orc.int8_to_float(g["codes"])
    assert out.tobytes() == g["table"].tobytes()
    assert out[0] == -1.0 and out[-1] == 1.0 and out[128] == 0.0


def test_am_golden(orc, golden_dir):
    g = np.load(os.path.join(golden_dir, "am_golden.npz"))
    am = orc.quad_am_demod(g["z"])
    assert np.all(np.abs(am - g["am"]) <= 1e-6 * g["am"] + 1e-30)
    assert list(am[:4]) == [0.0, 1.0, 1.0, 5.0]


def test_chain_golden_and_cpu_baseline(orc, golden_dir):
    g = np.load(os.path.join(golden_dir, "chain_golden.npz"))
    n_out = len(g["am"])
    for threads in (1, 3):
        am = orc.chain_i8_fc_am_f32(g["taps"], g["iq"], 1, n_out, threads=threads)
        assert np.all(np.abs(am - g["am"]) <= 1e-6 * g["bound"]), threads


def test_cpu_baseline_decimating(orc):
    rng = np.random.default_rng(3)
    taps = orc.lowpass_taps(1023, 0.04, "blackman")
    D, n_out = 10, 500
    x = (rng.standard_normal((n_out - 1) * D + 1023) + 1j * rng.standard_normal((n_out - 1) * D + 1023))
    x = x.astype(np.complex64)
    y, bound = orc.fir_f64(taps, x, D, n_out)
    am = orc.chain_fc_am_f32(taps, x, D, n_out, threads=2)
    assert np.all(np.abs(am - np.abs(y)) <= 1e-6 * bound)


def test_synth_sources_deterministic(orc):
    a = orc.synth_iq_int8(0x5EED, 20e6, 1e3, 1.5e6, 1000, 64)
    b = orc.synth_iq_int8(0x5EED, 20e6, 1e3, 1.5e6, 0, 1064)[2000:]
    assert a.tobytes() == b.tobytes()
    assert np.abs(a.astype(np.int32)).max() <= 127
    w = orc.synth_wideband_cf32(0xC3, 0.013, 0.31, 5, 16)
    assert np.all(np.isfinite(w.view(np.float32)))
