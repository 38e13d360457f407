"""The filter-graph boundary (gpusdrpipeline C++ ABI) on the GPU.

* the reference's own FIR / cosine known-answer tests, compiled as C++ against
  include/gpusdrpipeline (tests/cpp/abi_kats.cpp), run as a binary;
* the streaming contract replayed against the oracle's restatement
  (oracle.FirStreamModel: BaseSink.cpp:61-170 window, Fir.cpp:141-279 count/consume,
  partial reads of FirTests.cpp:96-221) under random chunking and random output capacities.
"""
import os
import subprocess

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIR_TOL = 1e-6


@pytest.fixture(scope="module")
def graph():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from gpusdr import graph as g
    return g


@pytest.fixture(scope="module")
def queue(graph):
    return graph.Queue(0)


def test_cpp_abi_kats():
    exe = os.path.join(REPO, "tests", "cpp", "_build", "abi_kats")
    if not os.path.exists(exe):
        subprocess.run(["make", "-s", "-C", os.path.join(REPO, "tests", "cpp")], check=True)
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0 and "ALL PASS" in r.stdout, r.stdout + r.stderr


def _drain(graph, queue, node, capacity, dtype):
    buf = graph.Buffer.create(queue, capacity)
    sl = buf.slice(0, capacity)
    sl.clear()
    node.read([sl])
    return sl.to_host(dtype)


@pytest.mark.parametrize("T,D,elem", [(2, 2, "c"), (127, 1, "c"), (63, 3, "f"), (1023, 10, "c"), (31, 4, "cc"),
                                      (64, 5, "cf"), (127, 1, "i8")])
def test_fir_streaming_matches_model(graph, queue, orc, T, D, elem):
    rng = np.random.default_rng(T * 10 + D)
    taps = orc.lowpass_taps(T, 0.4 / D) if T > 2 else np.array([0.5, 1.0], np.float32)
    if elem in ("cc", "cf"):
        taps = (taps * np.exp(0.2j * np.arange(T))).astype(np.complex64)
    et = {"c": graph.SAMPLE_FLOAT_COMPLEX, "cc": graph.SAMPLE_FLOAT_COMPLEX, "f": graph.SAMPLE_FLOAT,
          "cf": graph.SAMPLE_FLOAT, "i8": graph.SAMPLE_INT8_COMPLEX}[elem]
    node = graph.Node.fir(queue, taps, D, et)
    model = orc.FirStreamModel(taps, D)
    out_elem = 4 if (elem == "f") else 8
    out_dtype = np.float32 if elem == "f" else np.complex64
    total_out = 0
    for step in range(25):
        n = int(rng.integers(0, 3 * T + 50))
        if elem in ("c", "cc"):
            x = (rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64)
            node.push(x)
            model.push(x)
        elif elem in ("f", "cf"):
            x = rng.standard_normal(n).astype(np.float32)
            node.push(x)
            model.push(x)
        else:
            iq = rng.integers(-128, 128, size=2 * n).astype(np.int8)
            node.push(iq)
            model.push(orc.int8_to_float(iq).view(np.complex64))
        size, align = node.output_size()
        assert size == model.output_count() * out_elem
        assert align == 32 * out_elem
        cap = int(rng.integers(1, 40)) * out_elem
        y = _drain(graph, queue, node, cap, out_dtype)
        y64, bound = model.read(cap // out_elem)
        assert len(y) == len(y64)
        total_out += len(y)
        if len(y):
            assert np.all(np.abs(y.astype(np.complex128) - y64) <= FIR_TOL * bound + 1e-30), step
    assert total_out > 0


def test_elementwise_filters_bit_exact(graph, queue, orc):
    rng = np.random.default_rng(9)
    conv = graph.Node.int8_to_float(queue)
    am = graph.Node.quad_am_demod(queue)
    for _ in range(10):
        iq = rng.integers(-128, 128, size=int(rng.integers(1, 5000))).astype(np.int8)
        conv.push(iq)
        got = _drain(graph, queue, conv, 4 * len(iq) + 64, np.float32)
        assert got.tobytes() == orc.int8_to_float(iq).tobytes()
        z = (rng.standard_normal(len(iq)) * 5 + 1j * rng.standard_normal(len(iq))).astype(np.complex64)
        am.push(z)
        got = _drain(graph, queue, am, 4 * len(z), np.float32)
        assert got.tobytes() == orc.quad_am_demod(z).tobytes()


def test_cosine_source_phase_continuity(graph, queue, orc):
    src = graph.Node.cosine(queue, graph.SAMPLE_FLOAT_COMPLEX, 48000.0, 1234.5)
    assert src.output_size()[0] == 2 ** 64 - 1  # infinite source (CosineSource.cpp:59)
    delta = np.float32(2.0 * np.pi * 1234.5 / 48000.0)
    phi = np.float32(0.0)
    for n in (100, 37, 4096):
        z = _drain(graph, queue, src, 8 * n, np.complex64)
        assert len(z) == n
        phi_end = np.float32(phi + np.float32(n) * delta)
        ref = orc.cosine_c(float(phi), float(phi_end), n)
        assert np.max(np.abs(z - ref)) < 2e-5
        phi = np.float32(np.fmod(phi_end, np.float32(2.0 * np.pi)))


def test_json_nodes_and_out_of_scope(graph, queue):
    from gpusdr._native import lib
    import ctypes
    queue = graph.Queue.named("q0")  # the node's own stream for pushes and reads
    fir = graph.Node.from_json("Fir", '{"commandQueue": "q0", "taps": [0.5, 1.0], "tapType": "Float", '
                                      '"elementType": "FloatComplex", "decimation": 2}', queue)
    fir.push(np.array([0.1 + 0.2j, 0.3 + 0.4j, 0.5 + 0.6j, 0.7 + 0.8j, 0.9 + 0.9j], np.complex64))
    y = _drain(graph, queue, fir, 64, np.complex64)
    assert np.allclose(y, [0.35 + 0.5j, 0.95 + 1.1j], atol=1e-6)
    for name in ("HackRfSource", "AacWriter"):
        with pytest.raises(graph.GraphError) as e:
            graph.Node.from_json(name, '{"commandQueue": "q0"}')
        assert e.value.status == 8  # Status_NotFound
    with pytest.raises(graph.GraphError) as e:
        graph.Node.from_json("Fir", "{broken")
    assert e.value.status == 9  # Status_ParseError
    del lib, ctypes


@pytest.mark.parametrize("T,D", [(127, 1), (127, 3), (1023, 10)])
def test_stepping_driver_am_chain(graph, queue, orc, T, D):
    """Int8ToFloat -> Fir -> QuadAmDemod stepped by the SteppingDriver (SteppingDriver.cpp:193-366):
    the head is fed from outside the driver, every doFilter pulls one chunk through the chain, and
    the AM tail is drained between steps; the concatenated output equals the oracle chain over the
    whole stream (count rule Fir.cpp:178-186)."""
    rng = np.random.default_rng(T + D)
    taps = orc.lowpass_taps(T, 0.4 / D)
    conv = graph.Node.int8_to_float(queue)
    fir = graph.Node.fir(queue, taps, D, graph.SAMPLE_FLOAT_COMPLEX)
    am = graph.Node.quad_am_demod(queue)
    drv = graph.SteppingDriver()
    drv.connect(fir, 0, am, 0)  # downstream first: the tail must still be the AM node
    drv.connect(conv, 0, fir, 0)
    for node, name in ((conv, "int8ToFloat"), (fir, "fir"), (am, "amDemod")):
        drv.setup_node(node, name)
    assert drv.node_name(fir) == "fir"
    model = orc.FirStreamModel(taps, D)
    got, want, bounds = [], [], []
    for step in range(12):
        n = int(rng.integers(1, 200_000))
        iq = rng.integers(-128, 128, size=2 * n).astype(np.int8)
        conv.push(iq)
        model.push(orc.int8_to_float(iq).view(np.complex64))
        expect = model.output_count()
        for _ in range(64):  # a step moves at most the preferred 1 MiB per edge
            if am.output_size()[0] >= 4 * expect:
                break
            drv.do_filter()
        size, _ = am.output_size()
        assert size == 4 * expect
        got.append(_drain(graph, queue, am, max(size, 4), np.float32))
        y64, bound = model.read(model.output_count())
        want.append(np.abs(y64))
        bounds.append(bound)
    got, want, bound = np.concatenate(got), np.concatenate(want), np.concatenate(bounds)
    assert len(got) == len(want) > 0
    # AM of an FIR output: the FIR bound plus the sqrt rounding (AM_TOL relative)
    assert np.all(np.abs(got - want) <= FIR_TOL * bound + 1e-6 * want + 1e-30)



def test_multiply_filter_bit_exact(graph, queue, orc):
    """MultiplyCcc (Multiply.cpp:26-159): two ports filled unevenly, output = the common prefix,
    bit-exact against the oracle product; preferredInputBufferSize asks the lagging port for
    the difference."""
    queue = graph.Queue.named("qm")  # pushes and reads on the node's own stream
    mul = graph.Node.from_json("MultiplyCCC", '{"commandQueue": "qm"}', queue)
    rng = np.random.default_rng(4)
    a = (rng.standard_normal(5000) + 1j * rng.standard_normal(5000)).astype(np.complex64)
    b = (rng.standard_normal(5000) + 1j * rng.standard_normal(5000)).astype(np.complex64)
    assert mul.preferred_input_size(0) == 8192 * 8
    mul.push(a[:3000], port=0)
    mul.push(b[:1000], port=1)
    assert mul.preferred_input_size(0) == 0 and mul.preferred_input_size(1) == 2000 * 8
    assert mul.output_size()[0] == 1000 * 8
    got = [_drain(graph, queue, mul, 700 * 8, np.complex64)]
    mul.push(a[3000:], port=0)
    mul.push(b[1000:], port=1)
    got.append(_drain(graph, queue, mul, 5000 * 8, np.complex64))
    got = np.concatenate(got)
    assert got.tobytes() == orc.multiply_cc(a, b).tobytes()


def test_quad_fm_demod_filter(graph, queue, orc):
    """QuadFmDemod (QuadFmDemod.cpp:80-115): n inputs give n - 1 outputs, the last input is kept,
    so chunked reads equal the whole-stream discriminator; gain from QuadDemodFactory.h:111."""
    queue = graph.Queue.named("qf")
    fs, dev = 240000.0, 75000.0
    fm = graph.Node.from_json("QuadDemod", f'{{"commandQueue": "qf", "modulation": "fm", "sampleRate": {fs}, '
                                           f'"fskDeviation": {dev}}}', queue)
    gain = orc.fm_gain(fs, dev)
    rng = np.random.default_rng(8)
    n = 20000
    phase = np.cumsum(rng.uniform(-2.5, 2.5, n))
    z = (np.exp(1j * phase) * rng.uniform(0.5, 2.0, n)).astype(np.complex64)
    got, pos = [], 0
    for c in (1, 2, 777, 5000, 14220):
        fm.push(z[pos: pos + c])
        pos += c
        size, _ = fm.output_size()
        got.append(_drain(graph, queue, fm, max(size, 4), np.float32))
    got = np.concatenate(got)
    want = orc.quad_fm_demod_f64(z, gain)
    assert len(got) == n - 1
    # atan2f within 2 ulp of the float64 angle of the same float32 product
    assert np.all(np.abs(got - want) <= abs(gain) * (4 * np.spacing(np.float32(np.pi))) + 2 * np.spacing(np.abs(want).astype(np.float32)))


def test_frequency_shifter_fm_chain(graph, queue, orc):
    """The reference's FM front (RfToPcmAudioFactory.cpp:218-235): ComplexCosine -> MultiplyCcc
    port 1, IQ pushed into port 0 from outside, -> Fir (D=4) -> QuadFmDemod, stepped by the
    SteppingDriver. The driver pulls exactly the cosine samples the mixer lacks (the lagging port's
    preferred size), so the mixer sees one phase-continuous tone; the output is compared with the
    oracle chain over the whole stream."""
    queue = graph.Queue.named("qs")  # every node on one stream: pushes, kernels and reads ordered
    fs, shift, dev, D, T = 1.0e6, -150000.0, 75000.0, 4, 127
    cos = graph.Node.cosine(queue, graph.SAMPLE_FLOAT_COMPLEX, fs, shift)
    mul = graph.Node.from_json("MultiplyCCC", '{"commandQueue": "qs"}', queue)
    taps = orc.lowpass_taps(T, 0.1)
    fir = graph.Node.fir(queue, taps, D, graph.SAMPLE_FLOAT_COMPLEX)
    fm = graph.Node.from_json("QuadDemod", f'{{"commandQueue": "qs", "modulation": "fm", "sampleRate": {fs / D}, '
                                           f'"fskDeviation": {dev}}}', queue)
    drv = graph.SteppingDriver()
    drv.connect(cos, 0, mul, 1)
    drv.connect(mul, 0, fir, 0)
    drv.connect(fir, 0, fm, 0)
    rng = np.random.default_rng(21)
    n = 300000
    t = np.arange(n)
    msg = np.cumsum(0.3 * np.sin(2 * np.pi * 1e3 * t / fs))
    x = (np.exp(1j * (2 * np.pi * 150000.0 * t / fs + msg)) + 0.01 * rng.standard_normal(n)).astype(np.complex64)
    got, pos = [], 0
    for c in (50000, 1, 99999, 150000):
        mul.push(x[pos: pos + c], port=0)
        pos += c
        for _ in range(16):
            drv.do_filter()
        size, _ = fm.output_size()
        got.append(_drain(graph, queue, fm, max(size, 4), np.float32))
    got = np.concatenate(got)
    # oracle: the tone exp(j 2 pi shift i / fs), the mixer, the FIR in float64, the discriminator
    tone = np.exp(1j * 2 * np.pi * shift * t / fs)
    y, bound = orc.fir_f64(taps, (x * tone).astype(np.complex64), D)
    want = orc.fm_gain(fs / D, dev) * np.angle(y[1:] * np.conj(y[:-1]))
    assert len(got) == len(want)
    # The source forms phi_i = phi + i * step in float32 over a whole readOutput chunk before
    # reducing mod 2 pi (CosineSource.cpp:74-82, the reference's arithmetic, kept): with chunks of
    # up to 1 MiB the phase reaches ~1.2e5 rad, whose float spacing (7.8e-3 rad) is per-sample
    # phase noise of the tone. The FIR averages it; the discriminator keeps ~1e-3 rad of it
    # (a few outputs up to ~2e-2 where the spacing noise of neighbouring samples adds up).
    g = abs(orc.fm_gain(fs / D, dev))
    err = np.abs(got - want) / g
    assert np.median(err) <= 1e-3
    assert np.max(err) <= 5e-2, (int(np.argmax(err)), float(np.max(err)))


def _am_chain_graph(graph, queue, taps, D, qname="qg"):
    """int8 IQ -> Int8ToFloat -> Fir -> QuadAmDemod -> HipMemcpy (device -> host), all on one queue
    (`qname` names `queue`: the D2H filter is created from JSON, which names its queue - r06: the
    fixed-frame test passed "qf" but got a D2H on "qg", another stream, and its reference stream read
    one step's last AM sample before the AM kernel had written it, once in ~40 runs); the D2H filter
    is the graph tail the driver pulls through."""
    conv = graph.Node.int8_to_float(queue)
    fir = graph.Node.fir(queue, taps, D, graph.SAMPLE_FLOAT_COMPLEX)
    am = graph.Node.quad_am_demod(queue)
    d2h = graph.Node.from_json("HipMemcpy", '{"commandQueue": "%s", "from": "device", "to": "host"}' % qname, queue)
    drv = graph.SteppingDriver()
    drv.connect(conv, 0, fir, 0)
    drv.connect(fir, 0, am, 0)
    drv.connect(am, 0, d2h, 0)
    return conv, d2h, drv


def test_graph_stepping_matches_eager(graph, orc):
    """SteppingDriver steps of an int8 -> cf32 -> FIR -> AM chain fed fixed-size chunks: the
    graph-stepped driver (device work of each repeating chain state captured once, then replayed)
    gives the eager driver's output bit for bit, and most steps are replays."""
    queue = graph.Queue.named("qg")
    T, D, chunk, steps = 127, 2, 6000, 40
    taps = orc.lowpass_taps(T, 0.2)
    rng = np.random.default_rng(21)
    iq = rng.integers(-128, 128, size=2 * chunk * steps).astype(np.int8)
    outs = {}
    for mode in ("eager", "graphed"):
        conv, tail, drv = _am_chain_graph(graph, queue, taps, D)
        got = []
        for s in range(steps):
            conv.push(iq[2 * chunk * s: 2 * chunk * (s + 1)])
            drv.do_filter() if mode == "eager" else drv.do_filter_graphed(queue)
            got.append(_read_host(graph, queue, tail))
        outs[mode] = np.concatenate(got)
        if mode == "graphed":
            st = drv.graph_stats()
            assert st["replayed"] >= steps // 2 and st["captured"] >= 1, st
    assert outs["graphed"].tobytes() == outs["eager"].tobytes()
    x = orc.int8_to_float(iq).view(np.complex64)
    y64, bound = orc.fir_f64(taps, x, D, len(outs["eager"]))
    assert len(outs["eager"]) >= (chunk * steps - T) // D - chunk
    assert np.all(np.abs(outs["eager"] - np.abs(y64)) <= FIR_TOL * bound + 1e-30)


def _read_host(graph, queue, node):
    size, _ = node.output_size()
    if size == 0:
        return np.zeros(0, np.float32)
    buf = graph.Buffer.create_host(queue, size)
    sl = buf.slice(0, size)
    sl.clear()
    node.read([sl])
    return sl.to_host(np.float32)


def test_graph_stepping_falls_back_for_a_tone_source(graph, orc):
    """A chain with a CosineSource (its phase argument advances every step) is not replayable:
    every step runs plainly and the output equals the eager driver's."""
    queue = graph.Queue.named("qg")
    outs = {}
    for mode in ("eager", "graphed"):
        src = graph.Node.cosine(queue, graph.SAMPLE_FLOAT_COMPLEX, 48000.0, 1000.0)
        am = graph.Node.quad_am_demod(queue)
        d2h = graph.Node.from_json("HipMemcpy", '{"commandQueue": "qg", "from": "device", "to": "host"}', queue)
        drv = graph.SteppingDriver()
        drv.connect(src, 0, am, 0)
        drv.connect(am, 0, d2h, 0)
        got = []
        for _ in range(6):
            drv.do_filter() if mode == "eager" else drv.do_filter_graphed(queue)
            got.append(_read_host(graph, queue, d2h))
        outs[mode] = np.concatenate(got)
        if mode == "graphed":
            st = drv.graph_stats()
            assert st["captured"] == 0 and st["replayed"] == 0 and st["eager"] == 6, st
    assert outs["graphed"].tobytes() == outs["eager"].tobytes()
    assert len(outs["eager"]) > 0


def test_host_egress_sink_keeps_one_step_in_flight(graph, orc):
    """The host egress sink (reference AacFileWriter.cpp:267-280 without the codec, Waiter.cpp:34-50)
    at the tail of int8 -> cf32 -> FIR -> AM: the AM kernel writes into the sink's pinned host
    window; after each step everything but that step's bytes is in the host FIFO (one step in
    flight), flush() delivers the rest, and the stream equals the HipMemcpy D2H chain's bit for bit.
    Also reachable by JSON ("HostSink")."""
    queue = graph.Queue.named("qg")
    T, D, chunk, steps = 127, 2, 6000, 12
    taps = orc.lowpass_taps(T, 0.2)
    rng = np.random.default_rng(33)
    iq = rng.integers(-128, 128, size=2 * chunk * steps).astype(np.int8)
    # reference stream: the same chain ending in the D2H memcpy filter
    conv, tail, drv = _am_chain_graph(graph, queue, taps, D)
    ref, per_step = [], []
    for s in range(steps):
        conv.push(iq[2 * chunk * s: 2 * chunk * (s + 1)])
        drv.do_filter()
        ref.append(_read_host(graph, queue, tail))
        per_step.append(len(ref[-1]) * 4)
    ref = np.concatenate(ref)
    for make in (lambda: graph.Node.host_sink(queue),
                 lambda: graph.Node.from_json("HostSink", '{"commandQueue": "qg"}', queue)):
        conv = graph.Node.int8_to_float(queue)
        fir = graph.Node.fir(queue, taps, D)
        am = graph.Node.quad_am_demod(queue)
        sink = make()
        drv = graph.SteppingDriver()
        drv.connect(conv, 0, fir, 0)
        drv.connect(fir, 0, am, 0)
        drv.connect(am, 0, sink, 0)
        got, delivered = [], 0
        for s in range(steps):
            conv.push(iq[2 * chunk * s: 2 * chunk * (s + 1)])
            drv.do_filter()
            delivered += sink.host_available()
            got.append(sink.host_read(np.float32))
            assert delivered == sum(per_step[:s]), (s, delivered)  # step s still in flight
        sink.host_flush()
        got.append(sink.host_read(np.float32))
        got = np.concatenate(got)
        assert got.tobytes() == ref.tobytes()


def test_host_egress_sink_fixed_frame_reader(graph, orc):
    """A consumer that reads the host sink in fixed frames that do not line up with the step size
    (a codec's frame) rarely empties the FIFO; the consumed prefix is dropped as it grows (ADVICE
    r02), and the frames still concatenate to the D2H chain's stream bit for bit."""
    queue = graph.Queue.named("qf")
    T, D, chunk, steps, frame = 63, 2, 5000, 16, 4 * 777
    taps = orc.lowpass_taps(T, 0.2)
    rng = np.random.default_rng(34)
    iq = rng.integers(-128, 128, size=2 * chunk * steps).astype(np.int8)
    conv, tail, drv = _am_chain_graph(graph, queue, taps, D, "qf")
    ref = []
    for s in range(steps):
        conv.push(iq[2 * chunk * s: 2 * chunk * (s + 1)])
        drv.do_filter()
        ref.append(_read_host(graph, queue, tail))
    ref = np.concatenate(ref)
    conv = graph.Node.int8_to_float(queue)
    fir = graph.Node.fir(queue, taps, D)
    am = graph.Node.quad_am_demod(queue)
    sink = graph.Node.host_sink(queue)
    drv = graph.SteppingDriver()
    drv.connect(conv, 0, fir, 0)
    drv.connect(fir, 0, am, 0)
    drv.connect(am, 0, sink, 0)
    got = []
    for s in range(steps):
        conv.push(iq[2 * chunk * s: 2 * chunk * (s + 1)])
        drv.do_filter()
        while sink.host_available() >= frame:
            got.append(sink.host_read(np.float32, frame))
        assert sink.host_available() < frame
    sink.host_flush()
    got.append(sink.host_read(np.float32))
    assert np.concatenate(got).tobytes() == ref.tobytes()


def test_graph_replay_reports_ws_abort(graph, orc):
    """A wave-specialised kernel inside a graph-stepped chain that gives up a hand-off wait is not
    silent: with the spin limit at 0 (every unsatisfied wait aborts) the cf32 Fir node on the
    wave-specialised MFMA kernel (FFT off) aborts, and stepping the chain with a synchronisation
    between steps fails within a few steps (eager WS entry or the driver's post-replay check, ADVICE
    / VERDICT r02). With the limit restored and the count cleared, the same chain steps correctly."""
    import torch
    from gpusdr import ops
    queue = graph.Queue.named("qw")
    T, D, chunk = 1023, 10, 200_000
    taps = orc.lowpass_taps(T, 0.04)
    rng = np.random.default_rng(41)
    prev_pol = ops.set_kernel_policy(ops.POLICY_NO_FFT)
    prev_spin = ops.set_ws_spin_limit(0)
    try:
        ops.ws_aborts(reset=True)
        fir = graph.Node.fir(queue, taps, D, graph.SAMPLE_FLOAT_COMPLEX)
        am = graph.Node.quad_am_demod(queue)
        d2h = graph.Node.from_json("HipMemcpy", '{"commandQueue": "qw", "from": "device", "to": "host"}', queue)
        drv = graph.SteppingDriver()
        drv.connect(fir, 0, am, 0)
        drv.connect(am, 0, d2h, 0)
        failed = False
        for s in range(6):
            x = (rng.standard_normal(chunk) + 1j * rng.standard_normal(chunk)).astype(np.complex64)
            fir.push(x)
            try:
                drv.do_filter_graphed(queue)
            except graph.GraphError:
                failed = True
                break
            _read_host(graph, queue, d2h)
            torch.cuda.synchronize()
        assert failed, drv.graph_stats()
    finally:
        ops.set_ws_spin_limit(prev_spin)
        ops.set_kernel_policy(prev_pol)
        torch.cuda.synchronize()
        ops.ws_aborts(reset=True)  # never leak an abort into later tests


def test_replay_skips_host_step_and_matches_eager(graph, orc):
    """Replayed steps reinstate the host state the captured step left behind (window placement,
    used ranges, checkout flags) instead of re-running the step's host logic: over many steps of an
    int8 IQ -> Int8ToFloat -> Fir -> QuadAmDemod -> D2H chain at C3's filter shape (1023 taps,
    D = 10; the reference's two FIR/AM launches, fusion off) the graphed driver's output equals the
    eager driver's bit for bit, most steps are replays, and a replayed step's host time is below an
    eager step's (four launches and their node logic vs one graph launch)."""
    import time
    queue = graph.Queue.named("qr")
    T, D, chunk, steps = 1023, 10, 131_070, 40  # chunk a multiple of D: the consumed count repeats
    taps = orc.lowpass_taps(T, 0.04)
    rng = np.random.default_rng(43)
    xs = [rng.integers(-128, 128, size=2 * chunk).astype(np.int8) for _ in range(steps)]
    outs, host = {}, {}
    for mode in ("eager", "graphed"):
        conv = graph.Node.int8_to_float(queue)
        fir = graph.Node.fir(queue, taps, D, graph.SAMPLE_FLOAT_COMPLEX)
        am = graph.Node.quad_am_demod(queue)
        d2h = graph.Node.from_json("HipMemcpy", '{"commandQueue": "qr", "from": "device", "to": "host"}', queue)
        drv = graph.SteppingDriver()
        drv.set_fuse_fir_am(False)
        drv.connect(conv, 0, fir, 0)
        drv.connect(fir, 0, am, 0)
        drv.connect(am, 0, d2h, 0)
        got, times = [], []
        for s in range(steps):
            conv.push(xs[s])
            t0 = time.perf_counter()
            drv.do_filter() if mode == "eager" else drv.do_filter_graphed(queue)
            times.append(time.perf_counter() - t0)
            got.append(_read_host(graph, queue, d2h))
        outs[mode] = np.concatenate(got)
        host[mode] = float(np.median(times[steps // 2:]))
        if mode == "graphed":
            st = drv.graph_stats()
            assert st["replayed"] >= steps // 2, st
            # the step holds a D2H memcpy node: replayed through hipGraphLaunch, never as direct launches
            assert st["direct"] == 0, st
    assert outs["graphed"].tobytes() == outs["eager"].tobytes()
    assert len(outs["eager"]) > 0
    assert host["graphed"] < host["eager"], host


def test_fused_step_replays_as_direct_launch(graph, orc):
    """which replay path ran is observable. A steady-state fused Fir -> QuadAmDemod step into
    a DeviceSink captures as ONE kernel node and is replayed by launching that kernel with its captured
    parameters (no hipGraphLaunch): every replay is counted as direct; the chain's last Fir input window
    then holds exactly the unconsumed history, as eager stepping leaves it."""
    queue = graph.Queue.named("qdr")
    T, D, per, steps = 1023, 10, 8192, 24
    taps = orc.lowpass_taps(T, 0.04)
    rng = np.random.default_rng(7)
    left = {}
    for mode in ("eager", "graphed"):
        fir = graph.Node.fir(queue, taps, D, graph.SAMPLE_FLOAT_COMPLEX)
        am = graph.Node.quad_am_demod(queue)
        sink = graph.Node.from_json("DeviceSink", '{"commandQueue": "qdr", "preferredBytes": %d}' % (4 * per), queue)
        drv = graph.SteppingDriver()
        drv.connect(fir, 0, am, 0)
        drv.connect(am, 0, sink, 0)
        fir.push(np.zeros(T - 1, np.complex64))
        for s in range(steps):
            x = (rng.standard_normal(per * D) + 1j * rng.standard_normal(per * D)).astype(np.complex64)
            fir.push(x)
            drv.do_filter() if mode == "eager" else drv.do_filter_graphed(queue)
        queue.sync()
        left[mode] = fir.output_size()[0]
        st = drv.graph_stats()
        if mode == "graphed":
            assert st["replayed"] >= 4 and st["direct"] == st["replayed"], st
        else:
            assert st["replayed"] == 0 and st["direct"] == 0, st
    assert left["graphed"] == left["eager"]


@pytest.mark.parametrize("elem,T,D", [("c", 1023, 10), ("c", 127, 1), ("i8", 1023, 10), ("i8", 127, 1)])
def test_fused_fir_am_edge_matches_unfused(graph, orc, elem, T, D):
    """The driver steps a Fir (real taps) -> QuadAmDemod edge as ONE fused launch
    (gsdrFirFCAmDemod / gsdrInt8FirFCAmDemod): over random push sizes the fused and the reference's
    two-launch stepping (fusion off) both meet the float64 oracle chain, the AM node's window stays
    empty, and the stream lengths agree. (Not bit for bit: the two step the FIR in different launch
    sizes, and the FFT / matrix-core kernels' rounding depends on where a launch's blocks start.)"""
    queue = graph.Queue.named("qu")
    rng = np.random.default_rng(T + D + len(elem))
    taps = orc.lowpass_taps(T, 0.4 / D)
    et = graph.SAMPLE_FLOAT_COMPLEX if elem == "c" else graph.SAMPLE_INT8_COMPLEX
    sizes = [int(rng.integers(1, 300_000)) for _ in range(8)]
    if elem == "c":
        chunks = [(rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64) for n in sizes]
    else:
        chunks = [rng.integers(-128, 128, size=2 * n).astype(np.int8) for n in sizes]
    outs, stats = {}, {}
    for fuse in (False, True):
        fir = graph.Node.fir(queue, taps, D, et)
        am = graph.Node.quad_am_demod(queue)
        d2h = graph.Node.from_json("HipMemcpy", '{"commandQueue": "qu", "from": "device", "to": "host"}', queue)
        drv = graph.SteppingDriver()
        drv.set_fuse_fir_am(fuse)
        drv.connect(fir, 0, am, 0)
        drv.connect(am, 0, d2h, 0)
        got = []
        for c in chunks:
            fir.push(c)
            for _ in range(16):
                drv.do_filter()
                got.append(_read_host(graph, queue, d2h))
                if fir.output_size()[0] == 0 and am.output_size()[0] == 0:
                    break
        outs[fuse] = np.concatenate(got)
        stats[fuse] = drv.graph_stats()["fused"]
        if fuse:
            assert am.output_size()[0] == 0
    assert stats[False] == 0 and stats[True] > 0
    stream = np.concatenate(chunks)
    x = stream if elem == "c" else orc.int8_to_float(stream).view(np.complex64)
    assert len(outs[True]) == len(outs[False]) == (len(x) - (T - 1)) // D  # Fir.cpp:178-186 count rule
    y64, bound = orc.fir_f64(taps, x, D, len(outs[True]))
    for fuse in (True, False):
        assert np.all(np.abs(outs[fuse] - np.abs(y64)) <= FIR_TOL * bound + 1e-6 * np.abs(y64) + 1e-30), fuse


@pytest.mark.gpu
def test_device_sink_takes_one_preferred_chunk_per_step(graph, orc):
    """A DeviceSink (JSON "DeviceSink", preferredBytes) grows its window exactly to the request, as
    the reference's BaseSink does (BaseSink.cpp:75-77), so every fused Fir -> QuadAmDemod step moves
    exactly one preferred chunk: 8 192 envelopes (32 KiB, a whole number of allocation granules) per
    doFilter over ten chunks' worth of buffered outputs (the 2x headroom other sinks take would let
    the second step run two chunks)."""
    queue = graph.Queue.named("qds")
    T, D, per = 255, 4, 8192
    taps = orc.lowpass_taps(T, 0.1)
    fir = graph.Node.fir(queue, taps, D, graph.SAMPLE_FLOAT_COMPLEX)
    am = graph.Node.quad_am_demod(queue)
    sink = graph.Node.from_json("DeviceSink", '{"commandQueue": "qds", "preferredBytes": %d}' % (4 * per), queue)
    drv = graph.SteppingDriver()
    drv.connect(fir, 0, am, 0)
    drv.connect(am, 0, sink, 0)
    rng = np.random.default_rng(5)
    n = 10 * per * D + T - 1
    fir.push((rng.standard_normal(n) + 1j * rng.standard_normal(n)).astype(np.complex64))
    left = [fir.output_size()[0] // 8]
    for _ in range(10):
        drv.do_filter()
        left.append(fir.output_size()[0] // 8)
    queue.sync()
    assert left[0] == 10 * per
    assert [left[i] - left[i + 1] for i in range(10)] == [per] * 10
    assert drv.graph_stats()["fused"] == 10 and am.output_size()[0] == 0
