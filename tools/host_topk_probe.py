"""Host top-k T-band eigensolve (rbl.host.eig_topk) vs dsbevd at N = 512..896, kd = 32, under
BLAS thread limits 1-16 (threadpoolctl): picks the thread count for the convergence checks."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-randomized-block-lanczos_amd")]
import numpy as np
from threadpoolctl import threadpool_limits
from rbl import host

rng = np.random.default_rng(5)
for N in (512, 896):
    T = rng.standard_normal((33, N))
    for nt in (1, 2, 4, 8, 16):
        with threadpool_limits(limits=nt, user_api="blas"):
            for name, f in (("topk", lambda: host.eig_topk(T, 20)),
                            ("dsbevd", lambda: host.sort_eig_abs(*host.dsbev(T), 20))):
                f()
                t = time.perf_counter()
                for _ in range(5):
                    f()
                print(f"N={N} threads={nt:2d} {name:6s} {(time.perf_counter() - t) / 5 * 1e3:7.1f} ms", flush=True)
