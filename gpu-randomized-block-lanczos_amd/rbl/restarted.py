"""Restarted Lanczos with locking — Julia/restarted.jl (RBL_gpu_restarted, RBL_restarted).

Cycles of single-vector (b = 1) Lanczos on the device: partial reorth and reorth against
the locked Ritz vectors every third step (restarted.jl:53-57), local reorth every step, the
end-of-cycle reorth of the last two blocks (:100-102), then the T eigensolve on the host
(:103-104).  Ritz pairs whose residual bound |B_{m+1} s_m| < 1e-7 are locked (on the device)
in descending order until the first unconverged one, which restarts the next cycle
(:115-135); the Krylov size grows by 10 per cycle (:143).

Differences from the reference, by design:
  * V: the reference returns V = zeros(n, k) (restarted.jl:108, never assigned); here V holds
    the locked Ritz vectors, aligned with D;
  * a cycle's first block is reorthogonalised against the locked vectors before it is
    multiplied (the reference multiplies the un-reorthogonalised copy Qg_d, :41 vs :44): the
    two differ by the restart vector's locked components, which the previous cycle's reorth
    already removed to rounding level;
  * a cap on the cycles (max_cycles): the reference loops until k values converge.
"""
from __future__ import annotations

import numpy as np

from .host import dsbev
from .rbl_gpu import Context

LOCK_TOL = 1e-7   # restarted.jl:119 / :219


def _cycle(ctx: Context, b: int, kryl: int, first_flags: int):
    """restarted.jl:23-104 (lanczos_iteration_res) on the device; returns descending
    eigenvalues of T, its eigenvectors, the residual bounds and the block count m."""
    Ai, Bi, _ = ctx.step(1, first_flags)                  # :41-50
    cols = [Ai]
    Bs = [Bi]
    i = 2
    while i * b < kryl:                                    # :52
        flags = 3 if i % 3 == 0 else 0                     # :53-57
        Ai, Bi, _ = ctx.step(i, flags)                     # :58-81
        cols.append(Ai)
        Bs.append(Bi)
        i += 1
    m = i - 1                                              # blocks Q_1..Q_m
    ctx.reorth_last(m, 3)                                  # :100-102
    # T: insertA! of every A_i, insertB! of B_2..B_m (:84, :83-86 'if (i+1)*b < kryl_sz')
    T = np.zeros((b + 1, m * b))
    for j, A in enumerate(cols):
        for c in range(b):
            T[: b - c, j * b + c] = A[c:, c]
    for it in range(1, m):
        start = (it - 1) * b
        B = Bs[it - 1]
        for c in range(1, b + 1):
            T[b + 1 - c:, start + c - 1] = B[:c, c - 1]
    D, V = dsbev(T)                                        # :103
    res = Bs[-1] @ V[m * b - b:, ::-1]                     # :104 (descending order)
    return D[::-1].copy(), V[:, ::-1].copy(), res, m


def restarted(ctx: Context, k: int, *, kryl0: int = 100, omega=None, seed: int = 0,
              max_cycles: int = 60, tol: float = LOCK_TOL):
    """restarted.jl:106-146 on a loaded context.  Returns (D, V_local, cycles)."""
    b = 1
    max_blocks = kryl0 + 10 * max_cycles
    ctx.start(b, max_blocks, omega=omega, seed=seed)       # :112-113  Q = qr(A randn(n, 1))
    D = []
    count = 0
    kryl = kryl0
    cycles = 0
    first_flags = 2                                        # :41 reorth against the locked set
    while count < k and cycles < max_cycles:
        d, v, conv, m = _cycle(ctx, b, kryl, first_flags)
        ncomp = 0
        restart_s = None
        for i in range(d.size):                            # :116-137
            if count + ncomp >= k:
                break
            if np.linalg.norm(conv[:, i]) < tol:
                ncomp += 1
                ctx.lock(m, v[:, i:i + 1])                     # :121-126
                D.append(float(d[i]))
            else:
                restart_s = v[:, i:i + 1]                      # :131-132
                break
        if restart_s is None:  # nothing to restart from: the cycle's own start block again
            restart_s = np.zeros((m * b, b))
            restart_s[:b, :b] = np.eye(b)
        ctx.restart(m, restart_s)
        kryl += 10                                         # :143
        count += ncomp
        cycles += 1
    V = ctx.locked()
    return np.asarray(D), V, cycles


def RBL_gpu_restarted(A, k: int, *, device: int = 0, omega=None, seed: int = 0,
                      max_cycles: int = 60, return_cycles: bool = False):
    """Drop-in for RBL_gpu_restarted(A::SparseMatrixCSC{Float64}, k) (restarted.jl:106):
    the k largest (algebraic) eigenvalues, descending, by restarted b = 1 Lanczos with
    locking; V holds the locked Ritz vectors (the reference returns zeros)."""
    with Context(device) as ctx:
        ctx.set_matrix(A)
        D, V, cyc = restarted(ctx, k, kryl0=100, omega=omega, seed=seed, max_cycles=max_cycles)
    return (D, V, cyc) if return_cycles else (D, V)


def RBL_restarted(A, k: int, *, device: int = 0, omega=None, seed: int = 0,
                  max_cycles: int = 60, return_cycles: bool = False):
    """RBL_restarted(A, k) (restarted.jl:196-245, the CPU driver; sparse or dense A): the same
    cycle on the device with the CPU driver's first Krylov size, 80."""
    with Context(device) as ctx:
        ctx.set_matrix(A)
        D, V, cyc = restarted(ctx, k, kryl0=80, omega=omega, seed=seed, max_cycles=max_cycles)
    return (D, V, cyc) if return_cycles else (D, V)
