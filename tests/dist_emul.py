"""CPU restatement of the library's row-partitioned block Lanczos step over torch.distributed
(gloo), for the world_size > 1 tests (test infrastructure, like oracle/).

It drives the SAME host planning code the library uses (librbl_hip.so's
rbl_plan_row_partition / rbl_plan_halo / rbl_hashwindow_rows_host, which need no GPU) and
mirrors the library's data movement step for step (csrc/rbl_api.cpp):
  * setup_halo      — all-gather of every rank's need table -> the rows each rank gives;
  * halo_exchange   — grouped point-to-point Q rows (ncclSend/ncclRecv in the library);
  * gram            — local W^T X partial + all-reduce sum (ncclAllReduce);
  * tsqr            — CholQR2 on the all-reduced Gram (positive-diagonal R);
  * rbl_step order  — partial reorth (block CGS) at even i, local reorth, U = A Q_i -
                      Q_{i-1} B_i^T, A_i = Q_i^T U, U -= Q_i A_i, QR   (RBL_gpu.jl:164-184).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp
import torch
import torch.distributed as dist

from rbl import _lib


def allreduce(x: np.ndarray) -> np.ndarray:
    t = torch.from_numpy(np.ascontiguousarray(x))
    dist.all_reduce(t)
    return t.numpy()


def allgather_i64(x: np.ndarray) -> np.ndarray:
    P = dist.get_world_size()
    t = torch.from_numpy(np.ascontiguousarray(x, dtype=np.int64))
    out = [torch.zeros_like(t) for _ in range(P)]
    dist.all_gather(out, t)
    return np.stack([o.numpy() for o in out])


class DistRows:
    """One rank's rows of a symmetric matrix plus the halo plan (mirrors rbl_ctx)."""

    def __init__(self, n, rowptr_global=None, csr_global=None, hashwindow=None):
        P, me = dist.get_world_size(), dist.get_rank()
        self.n, self.P, self.me = n, P, me
        if hashwindow is not None:        # rbl_gen_matrix_hashwindow: uniform row split
            self.bounds = np.array([n * p // P for p in range(P + 1)], dtype=np.int64)
            r0, r1 = self.bounds[me], self.bounds[me + 1]
            W, dens, seed, plant = hashwindow
            rp, col, val = _lib.hashwindow_rows_host(n, W, dens, seed, plant, r0, r1)
        else:                             # rbl_set_matrix_csc: nnz-balanced partition
            self.bounds = _lib.plan_row_partition(csr_global.indptr, P)
            r0, r1 = self.bounds[me], self.bounds[me + 1]
            rp = csr_global.indptr[r0:r1 + 1] - csr_global.indptr[r0]
            sl = slice(csr_global.indptr[r0], csr_global.indptr[r1])
            col = csr_global.indices[sl].astype(np.int64)
            val = csr_global.data[sl]
        self.r0, self.r1 = int(r0), int(r1)
        self.A = sp.csr_matrix((val, col, rp), shape=(r1 - r0, n))
        # halo plan (upload_csr + setup_halo)
        lo, hi = _lib.plan_halo(rp, col, self.bounds)
        lo[me] = hi[me] = 0
        self.need_lo, self.need_hi = lo, hi
        table = allgather_i64(np.stack([lo, hi], axis=1).reshape(-1))   # [p][2q + {0,1}]
        self.give_lo = table[:, 2 * me].copy()
        self.give_hi = table[:, 2 * me + 1].copy()
        self.give_lo[me] = self.give_hi[me] = 0
        ext = [(self.r0, self.r1)] + [(lo[q], hi[q]) for q in range(P) if hi[q] > lo[q]]
        self.ext_lo = int(min(a for a, _ in ext))
        self.ext_hi = int(max(b for _, b in ext))
        self.A_ext = self.A[:, self.ext_lo:self.ext_hi]

    def halo(self, Q: np.ndarray) -> np.ndarray:
        b = Q.shape[1]
        ext = np.zeros((self.ext_hi - self.ext_lo, b))
        ext[self.r0 - self.ext_lo:self.r1 - self.ext_lo] = Q
        reqs, bufs = [], []
        for q in range(self.P):
            if q == self.me:
                continue
            if self.give_hi[q] > self.give_lo[q]:
                s = torch.from_numpy(np.ascontiguousarray(
                    Q[self.give_lo[q] - self.r0:self.give_hi[q] - self.r0]))
                reqs.append(dist.isend(s, q))
            if self.need_hi[q] > self.need_lo[q]:
                r = torch.zeros((int(self.need_hi[q] - self.need_lo[q]), b), dtype=torch.float64)
                reqs.append(dist.irecv(r, q))
                bufs.append((q, r))
        for r in reqs:
            r.wait()
        for q, r in bufs:
            ext[self.need_lo[q] - self.ext_lo:self.need_hi[q] - self.ext_lo] = r.numpy()
        return ext

    def spmm(self, Q: np.ndarray) -> np.ndarray:
        return self.A_ext @ self.halo(Q)


def gram(X: np.ndarray, Y: np.ndarray) -> np.ndarray:
    return allreduce(X.T @ Y)


def cholqr2(U: np.ndarray):
    """Two CholQR passes on all-reduced Grams (the library's tsqr, unshifted case)."""
    G = gram(U, U)
    R1 = np.linalg.cholesky(G).T
    Q = np.linalg.solve(R1.T, U.T).T
    G = gram(Q, Q)
    R2 = np.linalg.cholesky(G).T
    Q = np.linalg.solve(R2.T, Q.T).T
    return Q, R2 @ R1


def dist_lanczos_trace(M: DistRows, omega_local: np.ndarray, steps: int):
    """Per-step (A_i, B_i) of the first `steps` block steps on this rank's rows."""
    Q = []
    Qi, _ = cholqr2(M.spmm(omega_local))                   # rbl_start
    Q.append(Qi)
    tA, tB = [], []
    Bprev = None
    for i in range(1, steps + 1):
        Qi = Q[i - 1]
        Qm = Q[i - 2] if i >= 2 else None
        if i % 2 == 0 and i >= 3:                          # partial reorth (block CGS)
            Wm = np.hstack(Q[: i - 2])
            X = np.hstack([Qi, Qm])
            X -= Wm @ gram(Wm, X)
            b = Qi.shape[1]
            Qi[:] = X[:, :b]
            Qm[:] = X[:, b:]
        if i >= 2:                                         # local reorth (one projection)
            Qi -= Qm @ gram(Qm, Qi)
        U = M.spmm(Qi)
        if i >= 2:
            U -= Qm @ Bprev.T
        Ai = gram(Qi, U)
        U -= Qi @ Ai
        Qn, Bi = cholqr2(U)
        Q.append(Qn)
        tA.append(Ai)
        tB.append(Bi)
        Bprev = Bi
    return tA, tB, Q
