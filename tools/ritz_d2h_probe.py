"""Time rbl_ritz at C4a size (n = 1e7, k = 20, 38 blocks of b = 32) into host buffers of
different kinds: fresh np.zeros (first-touch page faults inside the copy), pre-touched; the
plain hipMemcpy into pageable memory (RBL_D2H_DIRECT=1) against the staged pinned copy."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-randomized-block-lanczos_amd")]
import numpy as np
import rbl
from rbl import _lib
from rbl._lib import lib, dptr

n, b, k = 10_000_000, 32, 20
with rbl.Context(0) as ctx:
    ctx.gen_hashwindow(n, 64, 0.7734, 20261015, np.array([100.0 * (2 * k + 1 - l) for l in range(1, 2 * k + 1)]))
    rbl.lanczos(ctx, k, b, check=False, ritz=False, max_steps=8)
    S = np.asfortranarray(np.random.default_rng(0).standard_normal((8 * b, k)))
    for kind, direct in [("zeros", 1), ("zeros", 0), ("touched", 1), ("touched", 0),
                         ("zeros", 1), ("zeros", 0), ("empty", 0)] + [("zeros", -t) for t in (4, 8, 12, 16)] * 2:
        if direct < 0:
            os.environ["RBL_D2H_THREADS"] = str(-direct)
        if direct > 0:
            os.environ["RBL_D2H_DIRECT"] = "1"
        else:
            os.environ.pop("RBL_D2H_DIRECT", None)
        V = np.empty((n, k), order="F") if kind == "empty" else np.zeros((n, k), order="F")
        if kind == "touched":
            V[::512] = 1.0  # one write per 4 KiB page
        ctx.synchronize()
        t = time.perf_counter()
        lib.rbl_ritz(ctx._h, 8, k, dptr(S), dptr(V))
        print(f"{kind:8s} direct={direct} rbl_ritz {1e3 * (time.perf_counter() - t):8.1f} ms", flush=True)
