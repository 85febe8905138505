"""Host-side helpers that stay on the CPU (north star: "the small T_j eigensolve on CPU").

Restates Julia/common.jl:9-65 for the product's host loop:
  * ``TBand``       — insertA!/insertB! (common.jl:9-26), kept as one preallocated lower band
                      instead of the reference's per-step ``T = [T insertA!(...)]`` reallocation
                      (RBL_gpu.jl:185);
  * ``dsbev``       — LAPACK dsbev(jobz='V', uplo='L') (common.jl:28-48), via SciPy's LAPACK
                      (dsbevd, the same eigenpairs to rounding, from N = 256 on: see below);
  * ``sort_eig_abs``  (common.jl:50-54) and ``check_convergence`` (common.jl:56-65).
"""
from __future__ import annotations

import os

import numpy as np
from scipy.linalg import lapack


class TBand:
    """Lower band storage (b+1) x N of the block tridiagonal T_j: T[1+r-c, c] = T_j[r, c]."""

    def __init__(self, b: int, max_blocks: int):
        self.b = b
        self.data = np.zeros((b + 1, b * max_blocks))
        self.nblocks = 0

    def insert_A(self, Ai: np.ndarray) -> None:
        """common.jl:9-17: column (i-1)b+j receives A_i[j:b, j] (tril)."""
        b, i = self.b, self.nblocks
        self.data[:, i * b:(i + 1) * b] = 0.0
        for j in range(b):
            self.data[: b - j, i * b + j] = Ai[j:, j]
        self.nblocks += 1

    def insert_B(self, Bi: np.ndarray, it: int) -> None:
        """common.jl:20-26: the last j rows of column (it-1)b+j receive B[0:j, j] (triu)."""
        b = self.b
        start = (it - 1) * b
        for j in range(1, b + 1):
            self.data[b + 1 - j:, start + j - 1] = Bi[:j, j - 1]

    def view(self) -> np.ndarray:
        return self.data[:, : self.nblocks * self.b]


# The reference calls LAPACK dsbev (QR iteration, common.jl:32-33).  From N = 256 on, dsbevd
# (divide and conquer on the same band reduction) returns the same eigenpairs to ~1e-13 and
# runs 3-6x faster (tools/host_eig_probe.py: N = 896, kd = 32: 1.11 s -> 0.18 s) — the host
# eigensolve is most of the time-to-k on slowly decaying spectra.  RBL_HOST_EIGEN=dsbev forces
# the reference's routine throughout.
_EIGEN = os.environ.get("RBL_HOST_EIGEN", "auto")
DSBEVD_MIN_N = 256


def dsbev(T: np.ndarray):
    """common.jl:36-48 — eigenpairs of the symmetric band matrix T (lower, kd = b)."""
    use_d = _EIGEN == "dsbevd" or (_EIGEN == "auto" and T.shape[1] >= DSBEVD_MIN_N)
    w, z, info = (lapack.dsbevd if use_d else lapack.dsbev)(T, compute_v=1, lower=1)
    if info != 0:
        raise np.linalg.LinAlgError(f"{'dsbevd' if use_d else 'dsbev'} info={info}")
    return w, z


def sort_eig_abs(D: np.ndarray, V: np.ndarray, k: int):
    """common.jl:50-54 — stable sort by |lambda| (Julia sortperm is stable); keep the top k."""
    perm = np.argsort(np.abs(D), kind="stable")[len(D) - k:]
    return D[perm], V[:, perm]


def check_convergence(B: np.ndarray, V: np.ndarray, b: int, k: int, tol: float) -> bool:
    """common.jl:56-65 — every ||B_{i+1} S[end-b+1:end, l]||_2 <= tol (absolute)."""
    Y = B @ V[V.shape[0] - b:, :k]
    return bool(np.all(np.linalg.norm(Y, axis=0) <= tol))
