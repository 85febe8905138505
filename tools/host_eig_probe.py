"""Host T-band eigensolver timing on this machine: LAPACK dsbev (the reference's routine,
common.jl:32-33) vs dsbevd (divide and conquer), kd = 32, N = i*b at the convergence checks."""
import time
import numpy as np
from scipy.linalg import lapack

lapack.dsbevd(np.ones((33, 64)), compute_v=1, lower=1)  # warm the BLAS thread pool
for N in [128, 256, 384, 512, 640, 768, 896, 1216]:
    T = np.random.default_rng(0).standard_normal((33, N))
    best = {}
    for name, fn in (("dsbev", lapack.dsbev), ("dsbevd", lapack.dsbevd)):
        ts = []
        for _ in range(3):
            t = time.perf_counter()
            fn(T, compute_v=1, lower=1)
            ts.append(time.perf_counter() - t)
        best[name] = min(ts) * 1e3
    print(f"N={N:5d}  dsbev {best['dsbev']:8.1f} ms  dsbevd {best['dsbevd']:8.1f} ms", flush=True)
