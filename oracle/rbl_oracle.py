"""CPU restatement of the reference Randomized Block Lanczos (RBL) — TEST INFRASTRUCTURE ONLY.

This module is the parity *oracle* for the MI355X HIP path.  It is imported only by
``tests/``, ``__graft_entry__.smoke()`` and the ``cpu_baseline`` leg of ``bench.py``;
the product path (``gpu-randomized-block-lanczos_amd/rbl``) never imports it and fails
loudly if the HIP library is missing.

It restates, in NumPy/SciPy, the *effective* semantics of

* ``Julia/RBL.jl:74-142``   (``lanczos_iteration`` / ``RBL`` / ``recover_eigvec``), and
* ``Julia/common.jl:9-65``  (``insertA!``, ``insertB!``, ``dsbev``, ``sort_eig_abs``,
  ``check_convergence``),

with the GPU driver's loop bound (``Julia/RBL_gpu.jl:211``: 1200) available through
``kryl_sz``.  Parity traps from SURVEY.md Appendix A are honoured:

* P1 — ``loc_reorth!`` (``RBL.jl:4-13``) is ONE projection without renormalisation:
  only the first iteration's in-place ``gemm!`` reaches the caller's block.
* P3 — Ritz coefficients are fp64 (``RBL.jl:61-71``), not the fp32 ``cu()`` path.
* P4 — ``qr_mode="posdiag"`` flips Householder signs so that ``R`` has a non-negative
  diagonal (the CholQR convention of the HIP path); ``"householder"`` keeps LAPACK's.
* P5 — the starting block ``Omega`` is an input (the reference draws it unseeded).
* P6 — non-convergence returns ``converged=False`` and best-effort Ritz pairs instead
  of the reference's BoundsError.
* P8 — partial reorth at even ``i`` touches ``Q_i`` and ``Q_{i-1}`` against
  ``Q_1..Q_{i-2}`` in ascending ``j`` (block MGS, ``RBL.jl:30-48``), before local reorth.

Pinning: ``tests/test_oracle.py`` runs the reference's own known-answer
suites (``Julia/Unit Testing/test.jl:16-50`` via ``mod_dec.jl``/``slow_dec.jl``/
``step_dec.jl``: relative eigenvalue-error norm < 1e-13).  Julia is absent from the
image, so no reference output can be generated; those suites are the pin.
"""
from __future__ import annotations

import numpy as np
import scipy.linalg
import scipy.sparse as sp
from scipy.linalg import lapack

RESIDUAL_TOL = 1e-7          # RBL.jl:109, RBL_gpu.jl:189 (absolute)
KRYL_SZ_CPU = 1400           # RBL.jl:133
KRYL_SZ_GPU = 1200           # RBL_gpu.jl:211


# ----------------------------------------------------------------------------------------
# common.jl restatement
# ----------------------------------------------------------------------------------------
def insertA(Ai: np.ndarray, b: int) -> np.ndarray:
    """common.jl:9-17 — a (b+1) x b lower-band slab holding tril(A_i)."""
    T = np.zeros((b + 1, b))
    nA = Ai.shape[1]
    for j in range(nA):
        T[: nA - j, j] = Ai[j:nA, j]
    return T


def insertB(Bi: np.ndarray, T: np.ndarray, b: int, it: int) -> None:
    """common.jl:20-26 — write triu(B_{it+1}) into the last rows of columns (it-1)b+1..it*b."""
    nB = Bi.shape[1]
    start = (it - 1) * b
    for j in range(1, nB + 1):
        T[T.shape[0] - j:, start + j - 1] = Bi[:j, j - 1]


def dsbev(T: np.ndarray):
    """common.jl:36-48 — LAPACK dsbev(jobz='V', uplo='L', kd=b) on the lower band T."""
    w, z, info = lapack.dsbev(T, compute_v=1, lower=1)
    if info != 0:  # the reference ignores info (common.jl:43-46); we surface it
        raise np.linalg.LinAlgError(f"dsbev info={info}")
    return w, z


def sort_eig_abs(D: np.ndarray, V: np.ndarray, k: int):
    """common.jl:50-54 — stable sort by |lambda| ascending, keep the top k (ascending)."""
    perm = np.argsort(np.abs(D), kind="stable")
    perm_k = perm[len(perm) - k:]
    return D[perm_k], V[:, perm_k]


def check_convergence(B: np.ndarray, V: np.ndarray, b: int, k: int, tol: float) -> bool:
    """common.jl:56-65 — ||B_{i+1} S[end-b+1:end, l]||_2 <= tol for every l."""
    Y = B @ V[V.shape[0] - b:, :]
    return bool(np.all(np.linalg.norm(Y[:, :k], axis=0) <= tol))


# ----------------------------------------------------------------------------------------
# RBL.jl restatement
# ----------------------------------------------------------------------------------------
def _qr(U: np.ndarray, mode: str):
    Q, R = np.linalg.qr(U, mode="reduced")     # LAPACK dgeqrf + dorgqr, as Julia's qr()
    if mode == "posdiag":
        s = np.sign(np.diag(R))
        s[s == 0] = 1.0
        Q = Q * s[None, :]
        R = R * s[:, None]
    return Q, R


def loc_reorth(U1: np.ndarray, U2: np.ndarray) -> None:
    """RBL.jl:4-13, effective semantics (P1): U1 -= U2 (U2^T U1), in place, once."""
    U1 -= U2 @ (U2.T @ U1)


def part_reorth(Q: list, mode: str = "mgs") -> None:
    """RBL.jl:30-48: reorthogonalise Q[i] and Q[i-1] against Q[1..i-2] (1-based).

    ``mode="mgs"`` is the reference's ascending-j block MGS; ``"cgs"`` is one block-CGS
    projection against all j at once (the HIP path's batched form).  ``"cgs_blocked"`` is the
    same CGS projection (every coefficient from the unmodified X) evaluated block by block, so
    that no (n x (i-2)b) copy of the basis is made: it differs from ``"cgs"`` only in the
    association of the sums, and lets the oracle run at n = 1e7 in a 62 GB container.
    """
    i = len(Q)
    if i < 3:
        return
    if mode == "mgs":
        for j in range(i - 2):
            Qj = Q[j]
            Q[i - 1] -= Qj @ (Qj.T @ Q[i - 1])
            Q[i - 2] -= Qj @ (Qj.T @ Q[i - 2])
    elif mode == "cgs_blocked":
        C = [(Q[j].T @ Q[i - 1], Q[j].T @ Q[i - 2]) for j in range(i - 2)]
        for j in range(i - 2):
            Q[i - 1] -= Q[j] @ C[j][0]
            Q[i - 2] -= Q[j] @ C[j][1]
    else:
        W = np.hstack(Q[: i - 2])
        X = np.hstack([Q[i - 1], Q[i - 2]])
        X -= W @ (W.T @ X)
        b = Q[0].shape[1]
        Q[i - 1][:] = X[:, :b]
        Q[i - 2][:] = X[:, b:]


def recover_eigvec(Q: list, S: np.ndarray, k: int) -> np.ndarray:
    """RBL.jl:61-71 — V = sum_j Q_j S[(j-1)b+1:jb, :] in fp64."""
    n, b = Q[0].shape
    V = np.zeros((n, k))
    nblk = S.shape[0] // b
    for j in range(nblk):
        V += Q[j] @ S[j * b:(j + 1) * b, :k]
    return V


class OracleResult:
    def __init__(self, D, V, iters, nblocks, converged, trace):
        self.D, self.V, self.iters, self.nblocks = D, V, iters, nblocks
        self.converged, self.trace = converged, trace

    def __iter__(self):               # allow  D, V = RBL(...)
        return iter((self.D, self.V))


def lanczos_iteration(A, k: int, b: int, kryl_sz: int, Qi: np.ndarray, *, qr_mode="householder",
                      reorth_mode="mgs", check=True, max_steps=None, trace=False):
    """RBL.jl:74-117 (CPU ``lanczos_iteration``), effective semantics.

    Returns (D descending |lambda|, S columns aligned, Q list, iters, converged, trace).
    """
    Q = [Qi]
    tr = {"A": [], "B": []} if trace else None
    U = A @ Qi                                            # :80
    Ai = Qi.T @ U                                         # :81
    U -= Qi @ Ai                                          # :82
    Qi, Bi = _qr(U, qr_mode)                              # :84-86
    if tr is not None:
        tr["A"].append(Ai.copy()); tr["B"].append(Bi.copy())
    T = insertA(Ai, b)                                    # :87
    insertB(Bi, T, b, 1)                                  # :88
    D = np.zeros(0); S = np.zeros((0, 0))
    converged = False
    i = 1
    while i * b < kryl_sz:                                # :90
        if max_steps is not None and i >= max_steps:
            break
        i += 1
        Q.append(Qi)                                      # :92
        if i % 2 == 0:                                    # :93-95
            part_reorth(Q, reorth_mode)
        loc_reorth(Q[i - 1], Q[i - 2])                    # :96
        U = A @ Q[i - 1]                                  # :97
        U -= Q[i - 2] @ Bi.T                              # :98
        Ai = Q[i - 1].T @ U                               # :99
        U -= Q[i - 1] @ Ai                                # :101
        Qi, Bi = _qr(U, qr_mode)                          # :102-104
        if tr is not None:
            tr["A"].append(Ai.copy()); tr["B"].append(Bi.copy())
        T = np.hstack([T, insertA(Ai, b)])                # :105
        if check and (i * b > k) and (i % 4 == 0):       # :106
            D, S = dsbev(T)                               # :107
            D, S = sort_eig_abs(D, S, k)                  # :108
            if check_convergence(Bi, S, b, k, RESIDUAL_TOL):   # :109
                converged = True
                break
        insertB(Bi, T, b, i)                              # :113
    if tr is not None:
        tr["T"] = T
    return D[::-1].copy(), S[:, ::-1].copy(), Q, i, converged, tr


def RBL(A, k: int, b: int, *, omega=None, seed=None, kryl_sz=KRYL_SZ_CPU, qr_mode="householder",
        reorth_mode="mgs", check=True, max_steps=None, trace=False) -> OracleResult:
    """RBL.jl:119-142 — k largest-|lambda| eigenpairs of symmetric A with block size b."""
    n = A.shape[1]
    if omega is None:
        omega = np.random.default_rng(seed).standard_normal((n, b))
    Qi, _ = _qr(A @ np.asarray(omega, dtype=np.float64), qr_mode)   # :136-137
    D, S, Q, iters, conv, tr = lanczos_iteration(A, k, b, kryl_sz, Qi, qr_mode=qr_mode,
                                                 reorth_mode=reorth_mode, check=check,
                                                 max_steps=max_steps, trace=trace)
    V = recover_eigvec(Q, S, k) if S.size else np.zeros((n, 0))    # :140
    if tr is not None:
        tr["S"] = S
        tr["Q"] = Q
    return OracleResult(D, V, iters, len(Q), conv, tr)


def RBL_gpu_semantics(A, k, b, **kw) -> OracleResult:
    """RBL_gpu.jl:205-221 semantics: the same loop with max Krylov size 1200."""
    kw.setdefault("kryl_sz", KRYL_SZ_GPU)
    return RBL(A, k, b, **kw)


# ----------------------------------------------------------------------------------------
# Known-answer generators — Julia/Unit Testing/test.jl:16-50
# ----------------------------------------------------------------------------------------
def RBL_gpu_mixed(A, k: int, b: int, *, omega, kryl_sz=KRYL_SZ_GPU, qr_mode="posdiag",
                  reorth_mode="mgs", check=True, max_steps=None, trace=False) -> OracleResult:
    """RBL_gpu.jl:134-219 with FLOAT = Float32, DOUBLE = Float64: the GPU driver's
    mixed mode.  The Krylov blocks (Qg, Qg1, Qgpu) and their partial / local reorth are fp32
    (NumPy float32 GEMMs, as CUBLAS sgemm); A*Q, the 3-term update, A_i, QR and T are fp64
    on the widened blocks (copyto! Qg_d <- Qg, :172-173); each QR output enters the basis
    rounded to fp32 (:180-182).  Ritz vectors in fp64 from the fp32 blocks (P3: fp64 Ritz).
    """
    f32 = np.float32
    Qg_d, _ = _qr(A @ np.asarray(omega, dtype=np.float64), qr_mode)      # :213-214
    Qg = Qg_d.astype(f32)                                                 # :142
    Qgpu = [Qg.copy()]                                                    # :149-151
    tr = {"A": [], "B": []} if trace else None
    U = A @ Qg_d                                                          # :152
    Ai = Qg_d.T @ U                                                       # :153
    U -= Qg_d @ Ai                                                        # :154
    Qn, Bi = _qr(U, qr_mode)                                              # :155, 159
    Qg1 = Qg_d.astype(f32)                                                # :156
    Qg_d = Qn
    Qg = Qg_d.astype(f32)                                                 # :157-158
    if tr is not None:
        tr["A"].append(Ai.copy()); tr["B"].append(Bi.copy())
    T = insertA(Ai, b)                                                    # :160
    insertB(Bi, T, b, 1)                                                  # :161
    D = np.zeros(0); S = np.zeros((0, 0))
    converged = False
    i = 1
    while i * b < kryl_sz:                                                # :162
        if max_steps is not None and i >= max_steps:
            break
        i += 1
        if i % 2 == 0 and i >= 3:                                         # :164-166, 59-81
            if reorth_mode == "mgs":
                for j in range(i - 2):
                    Wj = Qgpu[j]
                    Qg -= Wj @ (Wj.T @ Qg)
                    Qg1 -= Wj @ (Wj.T @ Qg1)
            else:
                W = np.hstack(Qgpu[: i - 2])
                X = np.hstack([Qg, Qg1])
                X -= W @ (W.T @ X)
                Qg[:] = X[:, :b]
                Qg1[:] = X[:, b:]
            Qgpu[i - 2] = Qg1.copy()                                      # :76, 78
        Qg -= Qg1 @ (Qg1.T @ Qg)                                          # :167, 83-93 (P1)
        Qgpu.append(Qg.copy())                                            # :168-172
        Qg_d = Qg.astype(np.float64)                                      # :173
        Qg1_d = Qg1.astype(np.float64)                                    # :174
        U = A @ Qg_d                                                      # :176
        U -= Qg1_d @ Bi.T                                                 # :177
        Ai = Qg_d.T @ U                                                   # :178
        U -= Qg_d @ Ai                                                    # :179
        Qn, Bi = _qr(U, qr_mode)                                          # :180, 184
        Qg1 = Qg_d.astype(f32)                                            # :181
        Qg_d = Qn
        Qg = Qg_d.astype(f32)                                             # :182-183
        if tr is not None:
            tr["A"].append(Ai.copy()); tr["B"].append(Bi.copy())
        T = np.hstack([T, insertA(Ai, b)])                                # :185
        if check and (i * b > k) and (i % 4 == 0):                       # :186
            D, S = dsbev(T)
            D, S = sort_eig_abs(D, S, k)
            if check_convergence(Bi, S, b, k, RESIDUAL_TOL):
                converged = True
                break
        insertB(Bi, T, b, i)                                              # :193
    D = D[::-1].copy()
    S = S[:, ::-1].copy()
    Qlist = [q.astype(np.float64) for q in Qgpu]
    V = recover_eigvec(Qlist, S, k) if S.size else np.zeros((A.shape[0], 0))
    if tr is not None:
        tr["T"] = T
        tr["S"] = S
    return OracleResult(D, V, i, len(Qgpu), converged, tr)


def _restart_cycle(A, b, kryl, Qg_d, locked, qr_mode):
    """restarted.jl:23-104 (lanczos_iteration_res), effective semantics with FLOAT = DOUBLE =
    Float64: the cycle's first block is reorthogonalised against the locked vectors in the
    basis copy (Qg) while Qg_d, un-reorthogonalised, is multiplied (:41, :44-48)."""
    def lock_reorth(X):                                   # restart_reorth_gpu! (:1-21)
        for l in locked:
            X -= l @ (l.T @ X)
    Qg = Qg_d.copy()
    lock_reorth(Qg)                                       # :41
    Qb = [Qg.copy()]                                      # :42-43
    U = A @ Qg_d                                          # :44
    Ai = Qg_d.T @ U                                       # :45
    U -= Qg_d @ Ai                                        # :46
    Qn, Bi = _qr(U, qr_mode)                              # :47, 51
    Qg1 = Qg_d.copy()                                     # :48
    Qg_d = Qn
    Qg = Qn.copy()                                        # :49-50
    cols, Bs = [Ai], [Bi]
    i = 2
    while i * b < kryl:                                   # :54
        if i % 3 == 0:                                    # :55-59
            lock_reorth(Qg1)
            lock_reorth(Qg)
            for j in range(i - 2):                        # hybrid_part_reorth! (RBL_gpu.jl:59-81)
                Wj = Qb[j]
                Qg -= Wj @ (Wj.T @ Qg)
                Qg1 -= Wj @ (Wj.T @ Qg1)
            Qb[i - 2] = Qg1.copy()
        Qg -= Qg1 @ (Qg1.T @ Qg)                          # :60 (P1)
        Qb.append(Qg.copy())                              # :61-64
        Qg_d = Qg.copy()
        Qg1_d = Qg1.copy()
        U = A @ Qg_d                                      # :67
        U -= Qg1_d @ Bi.T                                 # :68
        Ai = Qg_d.T @ U                                   # :69
        U -= Qg_d @ Ai                                    # :70
        Qn, Bi = _qr(U, qr_mode)                          # :71-75
        Qg1 = Qg_d.copy()
        Qg_d = Qn
        Qg = Qn.copy()
        cols.append(Ai)
        Bs.append(Bi)
        i += 1
    m = len(Qb)
    X1, X2 = Qb[m - 2], Qb[m - 1]                          # :100-102
    lock_reorth(X1)
    lock_reorth(X2)
    for j in range(m - 2):
        Wj = Qb[j]
        X2 -= Wj @ (Wj.T @ X2)
        X1 -= Wj @ (Wj.T @ X1)
    T = np.hstack([insertA(a, b) for a in cols])          # :52, :80
    for it in range(1, m):                                # insertB! unless (i+1)b >= kryl (:81-83)
        insertB(Bs[it - 1], T, b, it)
    D, V = dsbev(T)                                       # :103
    res = Bs[-1] @ V[m * b - b:, ::-1]                    # :104
    return D[::-1].copy(), V[:, ::-1].copy(), res, Qb


def RBL_restarted_semantics(A, k: int, *, omega, kryl0: int = 100, qr_mode="posdiag",
                            max_cycles: int = 60, tol: float = RESIDUAL_TOL):
    """restarted.jl:106-146 (RBL_gpu_restarted; kryl0 = 80 gives RBL_restarted, :196-245):
    b = 1 Lanczos cycles with locking.  Returns (D, locked vectors, cycles)."""
    b = 1
    Qg_d, _ = _qr(A @ np.asarray(omega, dtype=np.float64), qr_mode)     # :112-113
    locked, D = [], []
    count, kryl, cycles = 0, kryl0, 0
    while count < k and cycles < max_cycles:
        d, v, conv, Qb = _restart_cycle(A, b, kryl, Qg_d, locked, qr_mode)
        ncomp = 0
        for i in range(d.size):                                          # :116-137
            if count + ncomp >= k:
                break
            if np.linalg.norm(conv[:, i]) < tol:
                ncomp += 1
                locked.append(recover_eigvec(Qb, v[:, i:i + 1], 1))
                D.append(d[i])
            else:
                Qg_d = recover_eigvec(Qb, v[:, i:i + 1], 1)
                break
        kryl += 10
        count += ncomp
        cycles += 1
    V = np.hstack(locked) if locked else np.zeros((A.shape[0], 0))
    return np.asarray(D), V, cycles


def moderate_decay_matrix(n: int, k: int):
    """test.jl:17-28 — a_i = i(i+1)/2; expected a[n], a[n-1], ..."""
    a = np.cumsum(np.arange(1, n + 1, dtype=np.float64))
    return sp.diags(a).tocsr(), a[::-1][:k].copy()


def slow_decay_matrix(n: int, k: int):
    """test.jl:31-37 — a_i = i."""
    a = np.arange(1, n + 1, dtype=np.float64)
    return sp.diags(a).tocsr(), a[::-1][:k].copy()


def step_decay_matrix(n: int, k: int):
    """test.jl:40-50 — ones(n) except a[2k+1-i] = i*n for i=1..2k; expected a[1:k]."""
    a = np.ones(n)
    sz = 2 * k
    for i in range(1, sz + 1):
        a[sz - i] = i * n
    return sp.diags(a).tocsr(), a[:k].copy()


def rbl_residual(A, eig, k, b, **kw):
    """test.jl:10-14 — relative error vector (d - eig) ./ eig."""
    r = RBL(A, k, b, **kw)
    return (r.D - eig) / eig


KNOWN_ANSWER_SUITES = {
    # name: (generator, n values, k, b)  — mod_dec.jl/slow_dec.jl/step_dec.jl:3-7
    "moderate": (moderate_decay_matrix, list(range(100, 1000, 200)), 5, 5),
    "slow": (slow_decay_matrix, list(range(100, 1000, 200)), 5, 5),
    "step": (step_decay_matrix, list(range(100000, 1000000, 200000)), 5, 5),
}
KNOWN_ANSWER_TOL = 1e-13
