"""Diagnostic: RBL_gpu vs the oracle for dense / sparse A at several (n, b)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-randomized-block-lanczos_amd")]
import numpy as np
import scipy.sparse as sp
import rbl
from oracle import rbl_oracle as o

def case(n, b, dense, k=6):
    rng = np.random.default_rng(2)
    B = rng.standard_normal((n, n)) / np.sqrt(n)
    A = B + B.T + np.diag(np.r_[np.linspace(40, 30, 2 * k), np.zeros(n - 2 * k)])
    if not dense:
        A = sp.csr_matrix(A)
    omega = rng.standard_normal((n, b))
    ref = o.RBL_gpu_semantics(A, k, b, omega=omega, qr_mode="posdiag", reorth_mode="cgs")
    D, V, info = rbl.RBL_gpu(A, k, b, omega=omega, return_info=True)
    rel = (np.abs(D - ref.D) / np.abs(ref.D)).max()
    print(f"n={n} b={b} dense={dense}: iters gpu {info.iters} ref {ref.iters} rel {rel:.2e} status {info.status}", flush=True)

for n, b, dense in [(300, 48, False), (300, 48, True), (384, 64, False), (400, 64, False), (600, 96, False), (300, 40, False), (900, 144, False)]:
    case(n, b, dense)
