"""CPU restatement of the library's row-partitioned block Lanczos step over torch.distributed
(gloo), for the world_size > 1 tests (test infrastructure, like oracle/).

It drives the SAME host planning code the library uses (librbl_hip.so's
rbl_plan_row_partition / rbl_plan_halo / rbl_hashwindow_rows_host, which need no GPU) and
mirrors the library's data movement step for step (csrc/rbl_api.cpp):
  * setup_halo      — all-gather of every rank's need table -> the rows each rank gives;
  * halo_exchange   — grouped point-to-point Q rows (ncclSend/ncclRecv in the library);
  * PushPullRows    — the indexed halo with the push/pull split (RBL_OPT_HALO_PUSH);
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


class PushPullRows(DistRows):
    """The indexed halo with the push/pull split (RBL_OPT_HALO_PUSH; rbl_api.cpp prepare_push,
    push_products / push_exchange / push_finish): each off-rank product A[r,c] Q[c] is formed on
    the rank of the endpoint with the larger (row degree, smaller id) — Q[c] pulled into a ghost
    slot when that is c (tier 1), else A[c,r] Q[c] formed by c's owner from its own rows and the
    partial row r pushed (tier 2 dropped here).  Ghost slots = the tier-1 columns sorted by id;
    the push tier is tier 1 transposed; received partials are added in peer order."""

    def __init__(self, n, csr_global):
        super().__init__(n, csr_global=csr_global)
        P, me, r0, r1 = self.P, self.me, self.r0, self.r1
        A = self.A.tocsr()
        rp = A.indptr
        # global row degrees: every rank's slice padded to the longest, all-gathered
        w = int(max(self.bounds[q + 1] - self.bounds[q] for q in range(P)))
        mine = np.zeros(max(w, 1), np.int64)
        mine[:r1 - r0] = np.diff(rp)
        allg = allgather_i64(mine)
        deg = np.concatenate([allg[q][:self.bounds[q + 1] - self.bounds[q]] for q in range(P)])
        coo = A.tocoo()
        rows, cols, vals = coo.row.astype(np.int64), coo.col.astype(np.int64), coo.data
        grow = rows + r0
        own = (cols >= r0) & (cols < r1)
        up = (deg[cols] > deg[grow]) | ((deg[cols] == deg[grow]) & (cols < grow))
        t1, t2 = ~own & up, ~own & ~up
        owner = np.searchsorted(self.bounds, cols, side="right") - 1
        # symmetry check: my tier-2 entries towards q are q's tier-1 entries towards me
        cnt = np.concatenate([np.bincount(owner[t1], minlength=P), np.bincount(owner[t2], minlength=P)])
        table = allgather_i64(cnt)
        self.symmetric = all(table[p][P + q] == table[q][p] for p in range(P) for q in range(P))
        self.ghost = np.unique(cols[t1])                      # sorted: grouped by owner
        gown = np.searchsorted(self.bounds, self.ghost, side="right") - 1
        self.ghost_cnt = np.bincount(gown, minlength=P).astype(np.int64)
        self.ghost_off = np.concatenate([[0], np.cumsum(self.ghost_cnt)[:-1]])
        counts = allgather_i64(self.ghost_cnt)               # [p][q]: rows p asks of q
        self.send_cnt = counts[:, me].copy()
        self.send_cnt[me] = 0
        self.send_off = np.concatenate([[0], np.cumsum(self.send_cnt)[:-1]])
        got = self._exchange_rows(self.ghost.reshape(-1, 1).astype(np.float64),
                                  self.ghost_off, self.ghost_cnt, self.send_off, self.send_cnt, 1)
        self.send_idx = got[:, 0].astype(np.int64) - r0
        assert np.all((self.send_idx >= 0) & (self.send_idx < r1 - r0))
        slot = np.searchsorted(self.ghost, cols[t1])
        m = r1 - r0
        self.A_own = sp.csr_matrix((vals[own], (rows[own], cols[own] - r0)), shape=(m, m))
        self.A_pull = sp.csr_matrix((vals[t1], (rows[t1], slot)), shape=(m, self.ghost.size))
        self.A_push = self.A_pull.T.tocsr()                   # ghost slot x own row
        self.rows_moved = 2 * self.ghost.size                 # pulled + pushed, this rank

    def _exchange_rows(self, send_src, src_off, src_cnt, dst_off, dst_cnt, b):
        """Grouped point-to-point: rows src_off[q]:+src_cnt[q] of send_src go to q; dst_cnt[q]
        rows from q land at dst_off[q] (the library's Comm::exchange)."""
        out = np.zeros((int(dst_cnt.sum()), b))
        reqs, bufs = [], []
        for q in range(self.P):
            if q == self.me:
                continue
            if src_cnt[q]:
                reqs.append(dist.isend(torch.from_numpy(np.ascontiguousarray(
                    send_src[src_off[q]:src_off[q] + src_cnt[q]])), q))
            if dst_cnt[q]:
                r = torch.zeros((int(dst_cnt[q]), b), dtype=torch.float64)
                reqs.append(dist.irecv(r, q))
                bufs.append((q, r))
        for r in reqs:
            r.wait()
        for q, r in bufs:
            out[dst_off[q]:dst_off[q] + dst_cnt[q]] = r.numpy()
        return out

    def spmm(self, Q: np.ndarray) -> np.ndarray:
        b = Q.shape[1]
        # pull: the rows my peers asked for, received into my ghost slots
        ghosts = self._exchange_rows(Q[self.send_idx], self.send_off, self.send_cnt,
                                     self.ghost_off, self.ghost_cnt, b)
        U = self.A_own @ Q + self.A_pull @ ghosts
        # push: partial rows for my ghost slots to their owners; mine added in peer order
        partial = self.A_push @ Q
        got = self._exchange_rows(partial, self.ghost_off, self.ghost_cnt, self.send_off,
                                  self.send_cnt, b)
        np.add.at(U, self.send_idx, got)
        return U


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
