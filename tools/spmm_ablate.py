"""Diagnostics: time the LDS-window SpMM with compute or data loads ablated
(RBL_SPMM_ABLATE is read once per process, so run one mode per process)."""
import os, sys, time
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-randomized-block-lanczos_amd")]
import numpy as np
import rbl
n = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
ctx = rbl.Context(0)
ctx.gen_hashwindow(n, 64, 0.7734, 20261015, np.array([100.0 * (41 - l) for l in range(1, 41)]))
ctx.set_option(0, 1)
for rep in range(int(os.environ.get("REPS", "2"))):
    ctx.reset_timers()
    rbl.lanczos(ctx, 20, 32, seed=1, check=False, max_steps=8, ritz=False)
    ctx.synchronize()
t = ctx.timers()
print(os.environ.get("RBL_SPMM_ABLATE", "0"), "AQ ms per launch", t["AQ"] / 9, flush=True)
