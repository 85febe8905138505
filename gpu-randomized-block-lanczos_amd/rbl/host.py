"""Host-side helpers that stay on the CPU (north star: "the small T_j eigensolve on CPU").

Restates Julia/common.jl:9-65 for the product's host loop:
  * ``TBand``       — insertA!/insertB! (common.jl:9-26), kept as one preallocated lower band
                      instead of the reference's per-step ``T = [T insertA!(...)]`` reallocation
                      (RBL_gpu.jl:185);
  * ``dsbev``       — LAPACK dsbev(jobz='V', uplo='L') (common.jl:28-48), via SciPy's LAPACK
                      (dsbevd, the same eigenpairs to rounding, from N = 256 on: see below);
  * ``sort_eig_abs``  (common.jl:50-54) and ``check_convergence`` (common.jl:56-65);
  * ``fix_signs``   — not in the reference: each Ritz coefficient column's sign fixed so its
                      largest-magnitude entry is positive.  An eigenvector's sign is whatever
                      the LAPACK routine returns (dsbev, dsbevd and the top-k path may differ),
                      so V = [Q_1..Q_m] S is made deterministic whichever solver ran.
"""
from __future__ import annotations

import contextlib
import os

import numpy as np
from scipy.linalg import lapack

# NumPy advises transparent huge pages (madvise MADV_HUGEPAGE) for every array of >= 4 MiB.  With
# the kernel's THP defrag policy "madvise" (the MI355X box's), the first touch of such an array
# compacts memory synchronously, and on the box that stalls the GPU as well: a block step's
# band-tile SpMM ran 30 ms instead of 3.8 while the host eigensolve first touched its 4.7-MB
# dense matrix (N = 768), ~27 ms per first slow-spectrum run (profiles/r06_ttk_thp_stall.txt).
# The eigensolve's arrays (a few MB, used once) gain nothing from huge pages, so they are
# allocated without the advice; the Ritz vectors' large result array keeps it (its first touch
# with 4-KiB pages costs 60-90 ms more at C4a).
try:
    from numpy._core.multiarray import _set_madvise_hugepage as _np_madvise_hugepage
except ImportError:  # pragma: no cover - older NumPy layout
    try:
        from numpy.core.multiarray import _set_madvise_hugepage as _np_madvise_hugepage
    except ImportError:
        _np_madvise_hugepage = None


@contextlib.contextmanager
def small_pages():
    """NumPy arrays allocated inside use base pages (no MADV_HUGEPAGE); the setting is restored
    on exit."""
    if _np_madvise_hugepage is None:
        yield
        return
    prev = _np_madvise_hugepage(False)
    try:
        yield
    finally:
        _np_madvise_hugepage(prev)


class TBand:
    """Lower band storage (b+1) x N of the block tridiagonal T_j: T[1+r-c, c] = T_j[r, c]."""

    def __init__(self, b: int, max_blocks: int):
        self.b = b
        self.data = np.zeros((b + 1, b * max_blocks))
        self.nblocks = 0
        # one block's entries as flat index arrays: one 1-D scatter per block instead of b slice
        # assignments (~2.8 ms of host time per 38-step run at b = 32, between the GPU runs)
        ncols = b * max_blocks
        lr, lc = np.tril_indices(b)           # A_i[r, c], r >= c -> band (r - c, c)
        self._a = ((lr - lc) * ncols + lc, lr * b + lc, lc * b + lr)
        ur, uc = np.triu_indices(b)           # B_i[r, c], r <= c -> band (b - c + r, c)
        self._b = ((b - uc + ur) * ncols + uc, ur * b + uc, uc * b + ur)
        self._flat = self.data.reshape(-1)    # a view (C-contiguous)

    @staticmethod
    def _take(M: np.ndarray, src_c: np.ndarray, src_f: np.ndarray) -> np.ndarray:
        if M.flags.f_contiguous:
            return M.ravel(order="F")[src_f]
        return np.ascontiguousarray(M).ravel()[src_c]

    def insert_A(self, Ai: np.ndarray) -> None:
        """common.jl:9-17: column (i-1)b+j receives A_i[j:b, j] (tril)."""
        b, i = self.b, self.nblocks
        dst, src_c, src_f = self._a
        self.data[:, i * b:(i + 1) * b] = 0.0
        self._flat[dst + i * b] = self._take(np.asarray(Ai, dtype=np.float64), src_c, src_f)
        self.nblocks += 1

    def insert_B(self, Bi: np.ndarray, it: int) -> None:
        """common.jl:20-26: the last j rows of column (it-1)b+j receive B[0:j, j] (triu)."""
        dst, src_c, src_f = self._b
        self._flat[dst + (it - 1) * self.b] = self._take(np.asarray(Bi, dtype=np.float64), src_c, src_f)

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


# The loop needs only the k largest-|lambda| pairs of T (common.jl:50-54 keeps those), which lie
# among the k lowest and the k highest eigenvalues.  From N = 512 on (and N > 8k) the band is
# expanded to dense and reduced ONCE to tridiagonal form by the blocked dsytrd (the band
# reduction inside dsbev / dsbevd is unblocked), dstemr (MRRR) gives the 2k
# end pairs of the tridiagonal, and dormqr applies the reflectors to those 2k vectors only.
# Same eigenvalues as dsbev to ~1e-14 relative; vectors up to sign (tests/test_host_helpers.py).
# RBL_HOST_EIGEN=dsbev or dsbevd forces the whole-spectrum routine.  At these sizes one BLAS
# thread is fastest on the MI355X box's host (tools/host_topk_probe.py, N = 896: 31.6 ms on 1
# thread, 35-41 ms on 2-16), so the solve runs under a one-thread limit when threadpoolctl exists.
SUBSET_MIN_N = 512
try:
    from threadpoolctl import threadpool_limits as _tp_limits
except ImportError:  # pragma: no cover - the image ships it
    _tp_limits = None


def eig_topk(T: np.ndarray, k: int):
    """sort_eig_abs(*dsbev(T), k) (RBL_gpu.jl:187-188): the k largest-|lambda| eigenpairs of the
    band T (lower, kd = b), ascending |lambda|."""
    N = T.shape[1]
    with small_pages():
        if _EIGEN != "auto" or N < SUBSET_MIN_N or 8 * k >= N:
            return sort_eig_abs(*dsbev(T), k)
        if _tp_limits is not None:
            with _tp_limits(limits=1, user_api="blas"):
                return _eig_topk_dense(T, k)
        return _eig_topk_dense(T, k)


def _eig_topk_dense(T: np.ndarray, k: int):
    N = T.shape[1]
    from scipy.linalg import eigh_tridiagonal
    full = np.zeros((N, N), order="F")
    for r in range(T.shape[0]):
        idx = np.arange(N - r)
        full[idx + r, idx] = T[r, : N - r]
    c, d, e, tau, info = lapack.dsytrd(full, lower=1, lwork=64 * N, overwrite_a=1)
    if info != 0:
        raise np.linalg.LinAlgError(f"dsytrd info={info}")
    ends = [eigh_tridiagonal(d, e, select="i", select_range=rng, lapack_driver="stemr")
            for rng in ((0, k - 1), (N - k, N - 1))]
    Z = np.asfortranarray(np.hstack([ends[0][1], ends[1][1]]))
    # Q = diag(1, H(1)..H(N-1)): the reflectors sit below the subdiagonal (uplo = 'L')
    cq, _, info = lapack.dormqr("L", "N", c[1:, : N - 1], tau[: N - 1], Z[1:], lwork=128 * k,
                                overwrite_c=1)
    if info != 0:
        raise np.linalg.LinAlgError(f"dormqr info={info}")
    Z[1:] = cq
    return sort_eig_abs(np.concatenate([ends[0][0], ends[1][0]]), Z, k)


def sort_eig_abs(D: np.ndarray, V: np.ndarray, k: int):
    """common.jl:50-54 — stable sort by |lambda| (Julia sortperm is stable); keep the top k."""
    perm = np.argsort(np.abs(D), kind="stable")[len(D) - k:]
    return D[perm], V[:, perm]


def residual_norms(B: np.ndarray, V: np.ndarray, b: int, k: int) -> np.ndarray:
    """The k residual bounds ||B_{i+1} S[end-b+1:end, l]||_2 of common.jl:56-65."""
    return np.linalg.norm(B @ V[V.shape[0] - b:, :k], axis=0)


def speculation_depth(resid: list, tol: float, margin: float = 100.0, mid: float = 5.0) -> int:
    """How many steps rbl.lanczos(speculate="auto") enqueues ahead of the next convergence check,
    from the max residual bounds of the earlier checks.  The next bound is predicted as the last
    one times the last ratio (clamped to <= 1: geometric decay, the Lanczos rate; measured at C4a
    on the slow spectrum the prediction lands within 1.1x of the bound once the decay is steady,
    and overestimates it by up to 5x while the decay still accelerates).  Predicted above
    margin x tol: the check is expected to fail, so the 4 steps up to the next check (the next
    check's stride).  Above mid x tol (mid = 5: beyond the largest overestimate seen): 2 steps —
    an odd step and an even one, about the eigensolve's length at that size.  Above tol: 1 step
    (an odd step: no partial reorth, cheap to discard).  Otherwise, or with fewer than two earlier
    checks (no rate), none.  RBL_SPEC_MID=0 drops the 2-step tier (A/B)."""
    if len(resid) < 2 or not (resid[-1] > 0.0 and resid[-2] > 0.0):
        return 0
    pred = resid[-1] * min(1.0, resid[-1] / resid[-2])
    if pred > margin * tol:
        return 4
    if pred > mid * tol and os.environ.get("RBL_SPEC_MID", "1") != "0":
        return 2
    return 1 if pred > tol else 0


def check_convergence(B: np.ndarray, V: np.ndarray, b: int, k: int, tol: float) -> bool:
    """common.jl:56-65 — every ||B_{i+1} S[end-b+1:end, l]||_2 <= tol (absolute)."""
    return bool(np.all(residual_norms(B, V, b, k) <= tol))


def fix_signs(S: np.ndarray) -> np.ndarray:
    """Flip each column of S so that its largest-|.| entry (the first, on ties) is positive.
    V = [Q] S inherits the choice, so the Ritz vectors no longer depend on the eigensolver's
    sign convention (the reference returns whatever dsbev gives, common.jl:36-48)."""
    if S.size == 0:
        return S
    idx = np.argmax(np.abs(S), axis=0)
    sgn = np.where(S[idx, np.arange(S.shape[1])] < 0, -1.0, 1.0)
    return S * sgn
