#!/usr/bin/env python3
"""Time-to-k at C4a three times on one context, after one full-length run without Ritz vectors
(as bench.py measures it): the host split (start / fetch wait / eig / Ritz + D2H) per run — does
the first Ritz call pay one-off costs (the pinned staging slots)?"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-randomized-block-lanczos_amd")]
import numpy as np  # noqa: E402
import rbl  # noqa: E402

n, b, k = 10_000_000, 32, 20
plant = np.array([100.0 * (2 * k + 1 - l) for l in range(1, 2 * k + 1)])
if len(sys.argv) > 1 and sys.argv[1] == "slow":  # bench.py's slowly decaying spectrum
    plant = np.array([12.0 + 0.25 * (2 * k + 1 - l) for l in range(1, 2 * k + 1)])
with rbl.Context(0) as ctx:
    if "timers" in sys.argv[1:]:  # every stage timed, as bench.py's time-to-k runs
        ctx.set_option(0, 1)
    ctx.gen_hashwindow(n, 64, 0.7734, 20261015, plant)
    rbl.lanczos(ctx, k, b, check=False, ritz=False)  # as bench.py's timed runs: full-length, no Ritz
    for rep in range(3):
        ctx.synchronize()
        t = time.perf_counter()
        spec = os.environ.get("TTK_SPEC", "auto")
        spec = {"0": False, "auto": "auto", "1": True}.get(spec, spec)
        D, V, info = rbl.lanczos(ctx, k, b, seed=rep + 1, speculate=spec)
        dt = time.perf_counter() - t
        print(f"rep {rep}: {dt * 1e3:7.1f} ms iters={info.iters} start={info.start_ms:.1f} "
              f"fetch={info.fetch_ms:.1f} eig={info.eig_ms:.1f} ritz+d2h={info.ritz_ms:.1f} "
              f"spec={info.spec_steps}/{info.spec_wasted} resid={['%.1e' % r for r in info.resid]}",
              flush=True)
        del V
