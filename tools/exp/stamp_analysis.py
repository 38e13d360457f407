#!/usr/bin/env python3
"""Wave-span structure of an FFT-kernel stamp dump (fft_bench FFT_BENCH_STAMP_DUMP): per wave slot
(workgroup * 8 + wave) the shader-clock and 100 MHz stamps after the prologue and after its last
block. Prints the span distribution by wave index in the workgroup, by XCD (workgroup mod 8) and the
slowest / fastest workgroups, to tell a structural imbalance from noise.
Usage: stamp_analysis.py <dump.bin> [...]"""
import sys

import numpy as np

for path in sys.argv[1:]:
    st = np.fromfile(path, dtype=np.uint64).reshape(-1, 4).astype(np.float64)
    ok = (st[:, 3] > st[:, 1]) & (st[:, 2] > st[:, 0])
    idx = np.nonzero(ok)[0]
    span = (st[idx, 3] - st[idx, 1]) * 0.01  # us
    end = (st[idx, 3] - st[idx, 1].min()) * 0.01
    clk = (st[idx, 2] - st[idx, 0]) / (st[idx, 3] - st[idx, 1]) * 100.0
    wg, w = idx // 8, idx % 8
    print(f"== {path}: {len(idx)} waves, span us p0 {span.min():.1f} p10 {np.percentile(span, 10):.1f} "
          f"p50 {np.median(span):.1f} p90 {np.percentile(span, 90):.1f} max {span.max():.1f}; "
          f"last end {end.max():.1f}; clock MHz p50 {np.median(clk):.0f}")
    print("   by wave index in WG: " + " ".join(f"w{k}:{np.median(span[w == k]):.0f}" for k in range(8)))
    print("   by XCD (WG mod 8):   " + " ".join(f"x{k}:{np.median(span[wg % 8 == k]):.0f}/{span[wg % 8 == k].max():.0f}"
                                               for k in range(8)))
    wg_max = np.array([span[wg == g].max() for g in range(wg.max() + 1)])
    wg_med = np.array([np.median(span[wg == g]) for g in range(wg.max() + 1)])
    order = np.argsort(wg_max)
    print("   slowest WGs (max span): " + ", ".join(f"{g}:{wg_max[g]:.0f}" for g in order[-8:][::-1]))
    print("   fastest WGs (max span): " + ", ".join(f"{g}:{wg_max[g]:.0f}" for g in order[:8]))
    print(f"   per-WG max span p10 {np.percentile(wg_max, 10):.0f} p50 {np.median(wg_max):.0f} p90 "
          f"{np.percentile(wg_max, 90):.0f}; per-WG median p10 {np.percentile(wg_med, 10):.0f} p90 {np.percentile(wg_med, 90):.0f}")
    # within a SIMD (waves w and w + 4 of a WG are usually on one SIMD): spread between the pair
    pair = [abs(span[(wg == g) & (w == k)][0] - span[(wg == g) & (w == k + 4)][0])
            for g in range(wg.max() + 1) for k in range(4)
            if ((wg == g) & (w == k)).any() and ((wg == g) & (w == k + 4)).any()]
    print(f"   |span(w) - span(w+4)| median {np.median(pair):.0f} p90 {np.percentile(pair, 90):.0f}")
