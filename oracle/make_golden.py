"""Generate the committed golden fixtures in tests/golden/ (run in the dev container).

Independent of liborcl.so: every expected value here comes from plain numpy (float64),
so the fixtures pin the C oracle, which in turn pins the HIP kernels.

* kat_*.json   - the reference's own known-answer tests, transcribed as data:
                 tests/FirTests.cpp:8-94, tests/FirTests.cpp:96-221,
                 tests/CosineSourceTests.cpp:8-56.
* fir_golden.npz - FF/FC/CC/CF x T in {63,127,1023} x D in {1,2,10}: float32 inputs/taps,
                 float64 outputs from np.convolve(x, h[::-1], 'valid')[::D].
* am_golden.npz, int8_golden.npz, chain_golden.npz - AM envelope, the int8 scale table and
                 the int8 -> 127-tap FC FIR -> AM chain.

Usage: python oracle/make_golden.py   (writes tests/golden/ + MANIFEST.json with sha256)
"""
from __future__ import annotations

import hashlib
import json
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(os.path.dirname(HERE), "tests", "golden")


def lowpass(num_taps, cutoff, window="hamming"):
    n = np.arange(num_taps, dtype=np.float64) - (num_taps - 1) / 2.0
    h = 2.0 * cutoff * np.sinc(2.0 * cutoff * n)
    m = np.arange(num_taps, dtype=np.float64)
    if num_taps > 1:
        if window == "hamming":
            w = 0.54 - 0.46 * np.cos(2 * np.pi * m / (num_taps - 1))
        else:
            w = 0.42 - 0.5 * np.cos(2 * np.pi * m / (num_taps - 1)) + 0.08 * np.cos(4 * np.pi * m / (num_taps - 1))
        h = h * w
    return (h / h.sum()).astype(np.float32)


def fir_ref(taps, x, D, n_out):
    h = taps.astype(np.complex128 if np.iscomplexobj(taps) else np.float64)
    xx = x.astype(np.complex128 if np.iscomplexobj(x) else np.float64)
    y = np.convolve(xx, h[::-1], mode="valid")[::D][:n_out]
    bound = np.convolve(np.abs(xx), np.abs(h)[::-1], mode="valid")[::D][:n_out]
    return y, bound


def main():
    os.makedirs(OUT, exist_ok=True)
    rng = np.random.default_rng(0x5EED)

    # ---- reference KATs, transcribed --------------------------------------------------------
    kat1 = {
        "source": "/root/reference/tests/FirTests.cpp:8-94",
        "tapType": "Float", "elementType": "FloatComplex", "decimation": 2,
        "taps": [0.5, 1.0],
        "pushes": [[[0.1, 0.2], [0.3, 0.4], [0.5, 0.6]], [[0.7, 0.8], [0.9, 0.9]]],
        "reads": [{"capacity_elements": "2x getOutputDataSize", "expected": [[0.35, 0.5], [0.95, 1.1]]}],
        "abs_tol": 1e-3,
    }
    kat2 = {
        "source": "/root/reference/tests/FirTests.cpp:96-221",
        "tapType": "Float", "elementType": "FloatComplex", "decimation": 2,
        "taps": [0.5, 1.0, 0.25],
        "pushes": [[[0.1, 0.2], [0.3, 0.4], [0.5, 0.6], [0.7, 0.8], [0.1, 0.2], [0.3, 0.4], [0.5, 0.6], [0.7, 0.8]]],
        "reads": [{"capacity_elements": 1, "expected": [[0.475, 0.65]]},
                  {"capacity_elements": 2, "expected": [[0.975, 1.15], [0.475, 0.65]]}],
        "abs_tol": 1e-3,
    }
    kat_cos = {
        "source": "/root/reference/tests/CosineSourceTests.cpp:8-56",
        "sampleType": "FloatComplex", "sampleRate": 100.0, "frequency": 1.0,
        # 101 cf32 requested; the 32-byte aligned allocation gives 832 B = 104 elements and the
        # source fills the whole remaining capacity (ComplexCosineSource.cpp:70-72).
        "buffer_elements": 104, "checked_elements": 101,
        "expected_rule": "values[i] = (cos, sin)(2 pi i f / fs), |err| < 1e-4",
        "abs_tol": 1e-4,
    }
    for name, obj in (("kat_fir_two_commits.json", kat1), ("kat_fir_partial_reads.json", kat2),
                      ("kat_cosine_source.json", kat_cos)):
        with open(os.path.join(OUT, name), "w") as f:
            json.dump(obj, f, indent=1)

    # ---- FIR variants ----------------------------------------------------------------------
    arrays = {}
    n_out = 300
    for T in (63, 127, 1023):
        base = lowpass(T, 0.1 if T < 1000 else 0.04)
        for D in (1, 2, 10):
            n_in = (n_out - 1) * D + T
            for mode in ("FF", "FC", "CC", "CF"):
                tc = mode[0] == "C"
                xc = mode[1] == "C"
                if tc:
                    taps = (base * np.exp(1j * 0.3 * np.arange(T))).astype(np.complex64)
                else:
                    taps = base
                if xc:
                    x = (rng.standard_normal(n_in) + 1j * rng.standard_normal(n_in)).astype(np.complex64)
                else:
                    x = rng.standard_normal(n_in).astype(np.float32)
                y, bound = fir_ref(taps, x, D, n_out)
                key = f"{mode}_T{T}_D{D}"
                arrays[key + "_taps"] = taps
                arrays[key + "_x"] = x
                arrays[key + "_y"] = y
                arrays[key + "_bound"] = bound
    np.savez_compressed(os.path.join(OUT, "fir_golden.npz"), **arrays)

    # ---- AM envelope -------------------------------------------------------------------------
    z = (rng.standard_normal(4096) * 10 + 1j * rng.standard_normal(4096) * 10).astype(np.complex64)
    z[:4] = np.array([0, 1, 1j, -3 + 4j], dtype=np.complex64)
    am = np.abs(z.astype(np.complex128))
    np.savez_compressed(os.path.join(OUT, "am_golden.npz"), z=z, am=am)

    # ---- int8 scale table (float32 IEEE division is exact-rounded in numpy) -------------------
    codes = np.arange(-128, 128, dtype=np.int8)
    table = np.maximum(np.float32(-1.0), codes.astype(np.float32) / np.float32(127.0)).astype(np.float32)
    np.savez_compressed(os.path.join(OUT, "int8_golden.npz"), codes=codes, table=table)

    # ---- int8 IQ -> 127-tap FC FIR -> AM ---------------------------------------------------------
    taps = lowpass(127, 0.1)
    n_out = 2000
    n_in = n_out - 1 + len(taps)
    iq = rng.integers(-128, 128, size=2 * n_in, dtype=np.int16).astype(np.int8)
    xf = np.maximum(np.float32(-1.0), iq.astype(np.float32) / np.float32(127.0))
    x = (xf[0::2].astype(np.float64) + 1j * xf[1::2].astype(np.float64))
    y, bound = fir_ref(taps, x, 1, n_out)
    np.savez_compressed(os.path.join(OUT, "chain_golden.npz"), taps=taps, iq=iq, am=np.abs(y), bound=bound)

    manifest = {}
    for name in sorted(os.listdir(OUT)):
        if name == "MANIFEST.json":
            continue
        with open(os.path.join(OUT, name), "rb") as f:
            manifest[name] = hashlib.sha256(f.read()).hexdigest()
    manifest["_generator"] = "oracle/make_golden.py (numpy %s, seed 0x5EED)" % np.__version__
    with open(os.path.join(OUT, "MANIFEST.json"), "w") as f:
        json.dump(manifest, f, indent=1, sort_keys=True)
    print("wrote", OUT, {k: os.path.getsize(os.path.join(OUT, k)) for k in manifest if not k.startswith("_")})


if __name__ == "__main__":
    main()
