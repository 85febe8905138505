#!/usr/bin/env python3
"""Replicates bench.py's time-to-k sequence on one context to find what makes the slow-spectrum
run's rbl_ritz wait ~20-30 ms on an idle stream (RBL_RITZ_TRACE prints the split on stderr).
variant: bench   — planted full-length run, planted time-to-k (V kept), regenerate slow, start +
                   step 1, drop V, timed slow time-to-k (bench.py's order)
         noplant — the same without the planted time-to-k
         early   — the planted V dropped right after its run
         fresh   — the slow time-to-k in a fresh context (as the probe)
         keepv   — bench, but the planted V stays referenced (no munmap before the slow run)"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-randomized-block-lanczos_amd")]
import numpy as np  # noqa: E402
import rbl  # noqa: E402

variant = sys.argv[1]
n, b, k = 10_000_000, 32, 20
plant = np.array([100.0 * (2 * k + 1 - l) for l in range(1, 2 * k + 1)])
slow = np.array([12.0 + 0.25 * (2 * k + 1 - l) for l in range(1, 2 * k + 1)])
with rbl.Context(0) as ctx:
    ctx.set_option(0, 1)
    if variant != "fresh":
        ctx.gen_hashwindow(n, 64, 0.7734, 20261015, plant)
        rbl.lanczos(ctx, k, b, check=False, ritz=False)
        V = None
        if variant != "noplant":
            D, V, info = rbl.lanczos(ctx, k, b, seed=3)
            if variant == "early":
                V = None
    ctx.gen_hashwindow(n, 64, 0.7734, 20261015, slow)
    ctx.start(b, 38, seed=3)
    ctx.step(1, False)
    keep = V if variant == "keepv" else None
    V = None
    for rep in range(2):
        ctx.synchronize()
        t = time.perf_counter()
        D, V, info = rbl.lanczos(ctx, k, b, seed=3)
        dt = time.perf_counter() - t
        print(f"{variant} rep {rep}: {dt * 1e3:7.1f} ms iters={info.iters} eig={info.eig_ms:.1f} "
              f"ritz+d2h={info.ritz_ms:.1f}", flush=True)
        V = None
