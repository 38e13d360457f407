#!/usr/bin/env python3
"""r06: the host egress sink under a fixed-frame reader (tests/test_filter_graph.py::
test_host_egress_sink_fixed_frame_reader failed once, one float differing at a step boundary). Repeats that
test's two chains in one process and, per round, reports which chain's outputs differ from the float64
chain beyond the 1e-6 sum|h||x| bound and where (step, offset in the step)."""
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [os.path.join(REPO, "oracle"), REPO, os.path.join(REPO, "cuda-sdr_amd"), os.path.join(REPO, "tests")]
import oracle  # noqa: E402  (checker only)
from gpusdr import graph  # noqa: E402
from test_filter_graph import _am_chain_graph, _read_host  # noqa: E402

oracle.lib()
T, D, chunk, steps, frame = 63, 2, 5000, 16, 4 * 777
taps = oracle.lowpass_taps(T, 0.2)
queue = graph.Queue.named("qf")
graph.Queue.named("qg")  # the queue the old helper named
for rnd in range(int(sys.argv[1]) if len(sys.argv) > 1 else 20):
    rng = np.random.default_rng(34 + rnd)
    iq = rng.integers(-128, 128, size=2 * chunk * steps).astype(np.int8)
    conv, tail, drv = _am_chain_graph(graph, queue, taps, D, *sys.argv[2:3])
    ref, ref_steps = [], []
    for s in range(steps):
        conv.push(iq[2 * chunk * s: 2 * chunk * (s + 1)])
        drv.do_filter()
        ref.append(_read_host(graph, queue, tail))
        ref_steps.append(len(ref[-1]))
    ref = np.concatenate(ref)
    conv = graph.Node.int8_to_float(queue)
    fir = graph.Node.fir(queue, taps, D)
    am = graph.Node.quad_am_demod(queue)
    sink = graph.Node.host_sink(queue)
    drv = graph.SteppingDriver()
    drv.connect(conv, 0, fir, 0)
    drv.connect(fir, 0, am, 0)
    drv.connect(am, 0, sink, 0)
    got, avail = [], []
    for s in range(steps):
        conv.push(iq[2 * chunk * s: 2 * chunk * (s + 1)])
        drv.do_filter()
        avail.append(sink.host_available())
        while sink.host_available() >= frame:
            got.append(sink.host_read(np.float32, frame))
    sink.host_flush()
    got.append(sink.host_read(np.float32))
    got = np.concatenate(got)
    xc = oracle.int8_to_float(iq).view(np.complex64)
    y64, bound = oracle.fir_f64(taps, xc, D, len(ref))
    a64 = np.abs(y64)
    bad_ref = np.nonzero(~(np.abs(ref - a64) <= 1e-6 * bound + 1e-30))[0]
    n = min(len(got), len(ref))
    bad_got = np.nonzero(~(np.abs(got[:n] - a64[:n]) <= 1e-6 * bound[:n] + 1e-30))[0]
    diff = np.nonzero(got[:n].view(np.uint32) != ref[:n].view(np.uint32))[0]
    edges = np.cumsum(ref_steps)
    where = [(int(k), int(np.searchsorted(edges, k, side="right")), float(got[k]), float(ref[k]), float(a64[k]))
             for k in diff[:6]]
    print(f"round {rnd}: len got {len(got)} ref {len(ref)}, bit-diffs {diff.size}, ref over bound {bad_ref.size}, "
          f"sink over bound {bad_got.size}; diffs (k, step, got, ref, f64) {where}; ref per step {ref_steps[:3]}",
          flush=True)
