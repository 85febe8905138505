"""Diagnostics: does the fused local reorth (RBL_OPT_FUSE bit 2) run on several in-process
ranks?  Prints per-config max |dA| between fuse 3 and fuse 7 and the loc-reorth stage time."""
import threading
import numpy as np
import rbl
from rbl import _lib
from oracle import matgen

n, W, k, b = 150001, 64, 10, 32
plant = matgen.planted_spectrum(k)


def run(P, fuse):
    res = [None] * P
    if P == 1:
        with rbl.Context(0) as ctx:
            ctx.set_option(_lib.RBL_OPT_TIMERS, 1)
            ctx.set_option(_lib.RBL_OPT_FUSE, fuse)
            ctx.gen_hashwindow(n, W, 0.7734, 17, plant)
            _, _, info = rbl.lanczos(ctx, k, b, seed=9, check=False, max_steps=10, trace=True, ritz=False)
            return [(info, ctx.timers())]
    group = rbl.LocalGroup(P)

    def worker(r):
        with rbl.Context(0, group=group, rank=r) as ctx:
            ctx.set_option(_lib.RBL_OPT_TIMERS, 1)
            ctx.set_option(_lib.RBL_OPT_FUSE, fuse)
            ctx.gen_hashwindow(n, W, 0.7734, 17, plant)
            _, _, info = rbl.lanczos(ctx, k, b, seed=9, check=False, max_steps=10, trace=True, ritz=False)
            res[r] = (info, ctx.timers())
    th = [threading.Thread(target=worker, args=(r,)) for r in range(P)]
    [t.start() for t in th]
    [t.join() for t in th]
    group.close()
    return res


for P in (1, 3):
    a, c = run(P, 3), run(P, 7)
    d = max(np.abs(x - y).max() for x, y in zip(a[0][0].trace_A, c[0][0].trace_A))
    print(P, "max dA", d, "loc ms fuse3", a[0][1].get("loc reorth"), "fuse7", c[0][1].get("loc reorth"),
          "AQ", a[0][1].get("AQ"), c[0][1].get("AQ"), flush=True)
