"""Dense-A path throughput (rbl_set_matrix_dense): A*Q stage per launch on fp64 MFMA.
usage: python tools/dense_bench.py [n] [b]   (diagnostic)"""
import os, sys, time
sys.path[:0] = [os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gpu-randomized-block-lanczos_amd")]
import numpy as np
import rbl
from rbl import _lib
n = int(sys.argv[1]) if len(sys.argv) > 1 else 30000
b = int(sys.argv[2]) if len(sys.argv) > 2 else 32
rng = np.random.default_rng(0)
A = rng.standard_normal((n, n), dtype=np.float32).astype(np.float64)
A += A.T
t0 = time.perf_counter()
with rbl.Context(0) as ctx:
    ctx.set_matrix(A)
    up = time.perf_counter() - t0
    ctx.set_option(_lib.RBL_OPT_TIMERS, 1)
    steps = 16
    for rep in range(2):
        ctx.reset_timers()
        rbl.lanczos(ctx, 10, b, check=False, max_steps=steps, ritz=False)
        ctx.synchronize()
    t = ctx.timers()
launches = steps  # rbl_start + (steps - 1) block steps
ms = t["AQ"] / launches
flops = 2.0 * n * n * b
byts = 8.0 * n * n
print(f"dense n={n} b={b}: upload {up:.1f} s; A*Q {ms:.3f} ms per launch = "
      f"{flops / ms / 1e9:.1f} TF/s, {byts / ms / 1e6:.0f} GB/s of A; stages {t}")
