"""Host driver mirroring the reference's ``RBL_gpu(A, k, b)`` (Julia/RBL_gpu.jl:205-221).

The host keeps the loop control, the block-tridiagonal T_j and its LAPACK ``dsbev``
(Julia/common.jl), exactly as the north star asks; every n-sized operation — SpMM, local and
partial reorthogonalisation, tall-skinny QR, Ritz projection — runs in librbl_hip.so on the
MI355X.  Per step only the two b x b blocks A_i, B_{i+1} cross PCIe.

Semantics follow the GPU reference loop (RBL_gpu.jl:134-203):
  * max Krylov size 1200 (RBL_gpu.jl:211), step i runs while i*b < kryl_sz (:162);
  * partial reorth at even i (:164), local reorth every step (:167);
  * eigensolve + convergence test when i*b > k and i % 4 == 0 (:186-191), absolute 1e-7;
  * D returned in descending |lambda| (:202), V = [Q_1..Q_m] S in fp64 (RBL.jl:61-71, P3);
    each column of S (so each Ritz vector) signed so its largest coefficient is positive —
    LAPACK's eigenvector signs are arbitrary and differ between dsbev, dsbevd and the top-k
    path, so this makes V independent of the host eigensolver (parity is up to sign anyway).
Non-convergence (the reference's BoundsError) returns the last Ritz pairs
with ``info.converged = False`` and status RBL_WARN_NOT_CONVERGED.
"""
from __future__ import annotations

import math
import time
from dataclasses import dataclass, field

import numpy as np
import scipy.sparse as sp

from . import _lib
from ._lib import RBLError, dptr, i32ptr, i64ptr, lib, u8ptr
from .host import (TBand, dsbev, eig_topk, fix_signs,
                   residual_norms, sort_eig_abs, speculation_depth)

KRYL_SZ_GPU = 1200          # RBL_gpu.jl:211
RESIDUAL_TOL = 1e-7         # RBL_gpu.jl:189


class LocalGroup:
    """In-process rank group (rbl_local_group_create): the multi-rank code path with a
    host-staged transport instead of RCCL, so it runs with several ranks on one GPU."""

    def __init__(self, nranks: int):
        import ctypes as C
        self._h = C.c_void_p()
        st = lib.rbl_local_group_create(C.byref(self._h), nranks)
        if st < 0:
            raise RBLError(st, "rbl_local_group_create")
        self.nranks = nranks

    def close(self) -> None:
        if self._h:
            lib.rbl_local_group_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Context:
    """One librbl_hip context: one GPU, or one rank of a row-partitioned job."""

    def __init__(self, device: int = 0, nranks: int = 1, rank: int = 0,
                 unique_id: bytes | None = None, group: "LocalGroup | None" = None,
                 shm_path: str | None = None):
        """nranks == 1: a single-GPU context.  nranks > 1 with `unique_id`: one rank of an RCCL
        job (one process per GPU).  `group`: one rank of an in-process LocalGroup (each rank
        driven by its own thread; ranks may share a GPU).  `shm_path`: one rank of a
        process-per-rank job over the shared-memory transport (rbl_create_shm; ranks may share
        a GPU; every rank passes the same path, unique per job)."""
        import ctypes as C
        self._h = C.c_void_p()
        if group is not None:
            nranks = group.nranks
            st = lib.rbl_create_local(C.byref(self._h), device, group._h, rank)
        elif shm_path is not None:
            st = lib.rbl_create_shm(C.byref(self._h), device, nranks, rank, shm_path.encode())
        elif nranks == 1:
            st = lib.rbl_create(C.byref(self._h), device)
        else:
            uid = np.frombuffer(unique_id, dtype=np.uint8).copy()
            st = lib.rbl_create_dist(C.byref(self._h), device, nranks, rank, u8ptr(uid))
        self.nranks, self.rank, self.device = nranks, rank, device
        self._check(st, "rbl_create")
        self.b = None

    # -- plumbing -------------------------------------------------------------------------
    def _check(self, st: int, what: str) -> int:
        if st < 0:
            msg = lib.rbl_last_error(self._h).decode() if self._h else ""
            raise RBLError(st, f"{what}: {msg}")
        return st

    def close(self) -> None:
        if self._h:
            lib.rbl_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def set_option(self, opt: int, value: int) -> None:
        self._check(lib.rbl_set_option(self._h, opt, int(value)), "rbl_set_option")

    # -- matrix ---------------------------------------------------------------------------
    def set_matrix(self, A) -> None:
        """Upload A: a SciPy sparse matrix (any format) or a dense NumPy array
        (RBL_gpu(A::Matrix{Float64}): panel GEMM on fp64 MFMA; with several ranks each keeps
        the rows of the even split).  The sparse arrays passed are A's rows (CSR): for the
        symmetric A of RBL_gpu.jl:209 they are exactly Julia's SparseMatrixCSC arrays; for any
        other A the device then computes A Q, as cuSPARSE does on the CSC matrix (benchmark.jl:58
        runs an unsymmetric sprandn) and as julia/RBL_hip.jl does by transposing first."""
        if isinstance(A, np.ndarray):
            n = A.shape[0]
            if A.ndim != 2 or A.shape[1] != n:
                raise ValueError("dense A must be square")
            P, r = self.nranks, self.rank
            r0, r1 = (n * r) // P, (n * (r + 1)) // P
            self.set_matrix_dense_rows(n, r0, r1, A[r0:r1])
            return
        A = sp.csr_matrix(A)
        A.sort_indices()
        n = A.shape[1]
        rowptr = A.indptr.astype(np.int64)
        colind = A.indices.astype(np.int64)
        nzval = A.data.astype(np.float64)
        self._check(lib.rbl_set_matrix_csc(self._h, n, A.nnz, i64ptr(rowptr), i64ptr(colind),
                                           dptr(nzval), 0), "rbl_set_matrix_csc")

    def set_matrix_dense_rows(self, n, row_begin, row_end, A_rows) -> None:
        """Rows [row_begin,row_end) of a dense symmetric n x n matrix (rbl_set_matrix_dense)."""
        M = np.asfortranarray(A_rows, dtype=np.float64)
        if M.shape != (row_end - row_begin, n):
            raise ValueError("A_rows must be (row_end - row_begin) x n")
        self._check(lib.rbl_set_matrix_dense(self._h, n, row_begin, row_end, dptr(M),
                                             max(M.shape[0], 1)), "rbl_set_matrix_dense")

    def set_matrix_rows(self, n, row_begin, row_end, rowptr, colind, val, index_base=0) -> None:
        rowptr = np.ascontiguousarray(rowptr, dtype=np.int64)
        colind = np.ascontiguousarray(colind, dtype=np.int64)
        val = np.ascontiguousarray(val, dtype=np.float64)
        self._check(lib.rbl_set_matrix_csr_rows(self._h, n, row_begin, row_end, i64ptr(rowptr),
                                                i64ptr(colind), dptr(val), index_base),
                    "rbl_set_matrix_csr_rows")

    def gen_hashwindow(self, n: int, halfwidth: int, density: float, seed: int,
                       plant=None) -> None:
        plant = np.ascontiguousarray(plant if plant is not None else np.zeros(0), np.float64)
        self._check(lib.rbl_gen_matrix_hashwindow(self._h, n, halfwidth, density, seed,
                                                  plant.size, dptr(plant) if plant.size else None),
                    "rbl_gen_matrix_hashwindow")

    def gen_rmat(self, n: int, scale: int, edges: int, seed: int, plant=None,
                 a: float = 0.57, b: float = 0.19, c: float = 0.19) -> None:
        """Seeded symmetric R-MAT matrix generated on the device."""
        plant = np.ascontiguousarray(plant if plant is not None else np.zeros(0), np.float64)
        self._check(lib.rbl_gen_matrix_rmat(self._h, n, scale, edges, a, b, c, seed, plant.size,
                                            dptr(plant) if plant.size else None),
                    "rbl_gen_matrix_rmat")

    def gen_circuit(self, n: int = 1_585_478, seed: int = 20261015, plant=None,
                    width: int = 1259, p_edge: float = 0.95873) -> None:
        """Seeded circuit-like SPD matrix of G3_circuit's shape (BASELINE config 3), generated
        on the device (rbl_gen_matrix_circuit); the defaults give n and nnz of G3_circuit."""
        plant = np.ascontiguousarray(plant if plant is not None else np.zeros(0), np.float64)
        self._check(lib.rbl_gen_matrix_circuit(self._h, n, width, p_edge, seed, plant.size,
                                               dptr(plant) if plant.size else None),
                    "rbl_gen_matrix_circuit")

    def matrix_info(self):
        v = [np.zeros(1, np.int64) for _ in range(4)]
        self._check(lib.rbl_matrix_info(self._h, *[i64ptr(x) for x in v]), "rbl_matrix_info")
        n, r0, r1, nnz = (int(x[0]) for x in v)
        return n, r0, r1, nnz

    def row_ids(self) -> np.ndarray:
        """Original (generator) id of each local row (rbl_row_ids): r0..r1-1, or the inverse
        relabel of a matrix generated with RBL_OPT_RELABEL — the order of omega's and V's rows."""
        n, r0, r1, _ = self.matrix_info()
        ids = np.zeros(max(r1 - r0, 1), np.int64)
        self._check(lib.rbl_row_ids(self._h, i64ptr(ids)), "rbl_row_ids")
        return ids[: r1 - r0]

    def get_matrix_csr(self):
        n, r0, r1, nnz = self.matrix_info()
        rowptr = np.zeros(r1 - r0 + 1, np.int64)
        col = np.zeros(max(nnz, 1), np.int32)
        val = np.zeros(max(nnz, 1), np.float64)
        self._check(lib.rbl_get_matrix_csr(self._h, i64ptr(rowptr), i32ptr(col), dptr(val)),
                    "rbl_get_matrix_csr")
        return rowptr, col[:nnz], val[:nnz]

    def apply(self, X: np.ndarray) -> np.ndarray:
        """Y = A X on the device (local rows), through the same SpMM kernels as a step."""
        n, r0, r1, _ = self.matrix_info()
        X = np.asfortranarray(X, dtype=np.float64)
        b = X.shape[1]
        Y = np.zeros((r1 - r0, b), order="F")
        self._check(lib.rbl_apply(self._h, b, dptr(X), dptr(Y)), "rbl_apply")
        return Y

    def matrix_format(self) -> int:
        """0 CSR only, 1 band tiles, 2 packed band tiles, 3 half band tiles, 4 dense."""
        return self._check(lib.rbl_matrix_format(self._h), "rbl_matrix_format")

    def spmm_kernel_for(self, b: int) -> int:
        """The SpMM kernel rbl_step runs at block size b: 1 global-gather CSR, 2 LDS-window CSR,
        3 LDS-densified band, 4 dense panels, 5 band tiles, 6 segmented gather (the same ids
        RBL_OPT_SPMM_KERNEL takes)."""
        return self._check(lib.rbl_spmm_kernel_for(self._h, b), "rbl_spmm_kernel_for")

    # -- Krylov run -------------------------------------------------------------------------
    def start(self, b: int, max_blocks: int, omega=None, seed: int = 0, basis_bits: int = 64) -> None:
        """basis_bits 32: the mixed mode of RBL_gpu.jl with FLOAT = Float32 (fp32 Krylov blocks
        and reorth, fp64 A*Q / 3-term / QR / Ritz)."""
        om = None
        if omega is not None:
            om = np.asfortranarray(omega, dtype=np.float64)
        self._check(lib.rbl_start(self._h, b, max_blocks, basis_bits, dptr(om), seed), "rbl_start")
        self.b = b

    def step(self, i: int, part_reorth):
        """part_reorth: bool, or the flag word of rbl_step (bit 0 partial reorth, bit 1 the
        locked-vector reorth of the restarted variants)."""
        b = self.b
        A = np.zeros((b, b), order="F")
        B = np.zeros((b, b), order="F")
        st = self._check(lib.rbl_step(self._h, i, int(part_reorth), dptr(A), dptr(B)), "rbl_step")
        return A, B, st

    def step_async(self, i: int, part_reorth) -> None:
        """rbl_step_async: enqueue step i; A_i, B_{i+1} and its status come from fetch()."""
        self._check(lib.rbl_step_async(self._h, i, int(part_reorth)), "rbl_step_async")

    def fetch(self, i0: int, i1: int):
        """rbl_fetch: wait, then [(A_j, B_j, status_j) for j in i0..i1-1]."""
        b, m = self.b, i1 - i0
        A = np.zeros((m, b, b))
        B = np.zeros((m, b, b))
        st = np.zeros(m, np.int32)
        self._check(lib.rbl_fetch(self._h, i0, i1, dptr(A), dptr(B), i32ptr(st)), "rbl_fetch")
        # each b x b block arrives column-major
        return [(A[j].T.copy(order="F"), B[j].T.copy(order="F"), int(st[j])) for j in range(m)]

    # ---- restarted variants (restarted.jl) ----
    def restart(self, nblocks: int, S: np.ndarray) -> None:
        S = np.asfortranarray(S, dtype=np.float64)
        self._check(lib.rbl_restart(self._h, nblocks, dptr(S)), "rbl_restart")

    def lock(self, nblocks: int, S: np.ndarray) -> None:
        S = np.asfortranarray(S, dtype=np.float64)
        self._check(lib.rbl_lock(self._h, nblocks, S.shape[1], dptr(S)), "rbl_lock")

    def locked(self) -> np.ndarray:
        n, r0, r1, _ = self.matrix_info()
        L = lib.rbl_num_locked(self._h)
        V = np.zeros((r1 - r0, L), order="F")
        if L:
            self._check(lib.rbl_get_locked(self._h, dptr(V)), "rbl_get_locked")
        return V

    def reorth_last(self, nblocks: int, flags: int) -> None:
        self._check(lib.rbl_reorth_last(self._h, nblocks, flags), "rbl_reorth_last")

    def ritz(self, nblocks: int, k: int, S: np.ndarray) -> np.ndarray:
        n, r0, r1, _ = self.matrix_info()
        S = np.asfortranarray(S[: nblocks * self.b, :k], dtype=np.float64)
        V = np.zeros((r1 - r0, k), order="F")
        self._check(lib.rbl_ritz(self._h, nblocks, k, dptr(S), dptr(V)), "rbl_ritz")
        return V

    def get_block(self, j: int) -> np.ndarray:
        n, r0, r1, _ = self.matrix_info()
        Q = np.zeros((r1 - r0, self.b), order="F")
        self._check(lib.rbl_get_block(self._h, j, dptr(Q)), "rbl_get_block")
        return Q

    def num_blocks(self) -> int:
        return lib.rbl_num_blocks(self._h)

    def timers(self) -> dict:
        names = _lib.stage_names()
        ms = np.zeros(len(names))
        self._check(lib.rbl_timers(self._h, dptr(ms), len(names)), "rbl_timers")
        return dict(zip(names, ms.tolist()))

    def reset_timers(self) -> None:
        self._check(lib.rbl_reset_timers(self._h), "rbl_reset_timers")

    def device_memory(self) -> tuple:
        """(free, total) bytes of the context's GPU (rbl_device_memory)."""
        f, t = np.zeros(1, np.int64), np.zeros(1, np.int64)
        self._check(lib.rbl_device_memory(self._h, i64ptr(f), i64ptr(t)), "rbl_device_memory")
        return int(f[0]), int(t[0])

    def comm_info(self) -> dict:
        """Ranks as the transport counts them (RCCL: ncclCommCount), this rank, transport name."""
        import ctypes as C
        n, r = C.c_int(0), C.c_int(0)
        buf = C.create_string_buffer(32)
        self._check(lib.rbl_comm_info(self._h, C.byref(n), C.byref(r), buf, 32), "rbl_comm_info")
        out = {"nranks": n.value, "rank": r.value, "transport": buf.value.decode()}
        if out["transport"] == "rccl":
            out.update(rccl_version())
        return out

    def comm_stats(self, reset: bool = False, times: bool = False) -> dict:
        """Collectives this rank issued since the last reset (rbl_comm_stats): all-reduce
        calls / bytes, halo exchanges, bytes sent / received; and the halo plan of the matrix
        held (not reset): halo_push (the push/pull split runs, RBL_OPT_HALO_PUSH) and the Q rows
        per SpMM summed over ranks its setup predicted with the split / with the pull-all halo;
        with times=True also the time in the collectives (ns): host wall time inside the
        transport calls, and their hipEvent spans on the streams (recorded only while
        RBL_OPT_TIMERS is 1)."""
        out = np.zeros(12, np.int64)
        self._check(lib.rbl_comm_stats(self._h, i64ptr(out), 12, int(reset)), "rbl_comm_stats")
        keys = ("allreduce_calls", "allreduce_bytes", "exchange_calls", "send_bytes",
                "recv_bytes", "halo_push", "push_rows_pred", "pull_rows_pred")
        if times:  # (timings differ run to run: counts-only dicts compare across runs)
            keys += ("allreduce_host_ns", "exchange_host_ns", "allreduce_dev_ns", "exchange_dev_ns")
        return dict(zip(keys, (int(x) for x in out)))

    def path_stats(self, reset: bool = False) -> dict:
        """Which code path the steps took since the last reset (rbl_path_stats), counted as the
        work is issued: SpMM launches, those that applied the local-reorth update, separate
        local-reorth passes and Grams, the fused path's edge fix-ups, two-wave SpMM launches
        (variants build only), and rbl_ritz calls that took the row-piece form."""
        from . import _lib as L
        out = np.zeros(L.RBL_PATH_NSTATS, np.int64)
        self._check(lib.rbl_path_stats(self._h, i64ptr(out), L.RBL_PATH_NSTATS, int(reset)),
                    "rbl_path_stats")
        return dict(zip(("spmm", "spmm_loc_fused", "loc_separate", "loc_gram", "locfix_edges",
                         "locfix_rest", "spmm_two_wave", "ritz_pieces"), (int(x) for x in out)))

    def allgather(self, values) -> np.ndarray:
        """rbl_allgather_host: every rank's int64 values, shape (nranks, len(values)); ordered
        after the work enqueued on this context (a collective: every rank calls it)."""
        mine = np.ascontiguousarray(np.asarray(values, dtype=np.int64).ravel())
        out = np.zeros(self.nranks * mine.size, np.int64)
        self._check(lib.rbl_allgather_host(self._h, i64ptr(mine), i64ptr(out), mine.size),
                    "rbl_allgather_host")
        return out.reshape(self.nranks, mine.size)

    def synchronize(self) -> None:
        self._check(lib.rbl_synchronize(self._h), "rbl_synchronize")


@dataclass
class RBLInfo:
    iters: int = 0
    nblocks: int = 0
    converged: bool = False
    status: int = 0
    qr_shifted_steps: int = 0
    eig_ms: float = 0.0          # host T-band eigensolves (dsbev / dsbevd)
    fetch_ms: float = 0.0        # host waits in rbl_fetch (the GPU finishing enqueued steps)
    ritz_ms: float = 0.0         # host wall time of rbl_ritz (device work + D2H of V)
    start_ms: float = 0.0        # host wall time of rbl_start (A Omega + QR)
    enqueue_ms: float = 0.0      # host time inside rbl_step_async (enqueueing the steps)
    spec_steps: int = 0          # steps enqueued ahead of a convergence check (speculate)
    spec_wasted: int = 0         # of those, steps past the converging check (discarded)
    resid: list = field(default_factory=list)   # max residual bound at each check
    trace_A: list = field(default_factory=list)
    trace_B: list = field(default_factory=list)


def rccl_version() -> dict:
    """The RCCL the library's RCCL transport calls (rbl_rccl_version: ROCm's own, opened by path
    whatever copy the process loaded first): {"rccl_version": "2.27.7", "rccl_version_code":
    22707, "rccl_path": file}.  No GPU call."""
    import ctypes as C
    v = C.c_int(0)
    buf = C.create_string_buffer(512)
    st = lib.rbl_rccl_version(C.byref(v), buf, 512)
    if st != 0:
        raise RBLError(st, f"rbl_rccl_version: {buf.value.decode()}")
    code = v.value
    # NCCL_VERSION(X,Y,Z): X*10000 + Y*100 + Z from 2.9 on
    return {"rccl_version": f"{code // 10000}.{code // 100 % 100}.{code % 100}",
            "rccl_version_code": code, "rccl_path": buf.value.decode()}


def max_steps_for(kryl_sz: int, b: int) -> int:
    """Number of block steps the loop `while i*b < kryl_sz` can run (RBL_gpu.jl:162)."""
    return max(1, math.ceil(kryl_sz / b))


def lanczos(ctx: Context, k: int, b: int, *, kryl_sz: int = KRYL_SZ_GPU, omega=None, seed=0,
            check: bool = True, max_steps: int | None = None, tol: float = RESIDUAL_TOL,
            trace: bool = False, ritz: bool = True, basis_bits: int = 64,
            speculate: "bool | int | str" = "auto"):
    """RBL_gpu.jl:134-203 + :219 on an already-loaded context.  Returns (D, V_local, info)."""
    steps_cap = max_steps_for(kryl_sz, b)
    if max_steps is not None:
        steps_cap = min(steps_cap, max_steps)
    info = RBLInfo()
    t0 = time.perf_counter()
    ctx.start(b, steps_cap, omega=omega, seed=seed, basis_bits=basis_bits)
    info.start_ms = (time.perf_counter() - t0) * 1e3
    T = TBand(b, steps_cap)
    D = np.zeros(0)
    S = np.zeros((0, 0))

    def _record(A, B, st):
        if st == _lib.RBL_WARN_QR_SHIFTED:
            info.qr_shifted_steps += 1
        if trace:
            info.trace_A.append(A.copy())
            info.trace_B.append(B.copy())

    # Steps are enqueued without a host round trip (rbl_step_async) and fetched where the host
    # needs the T band: at a convergence check (:186) and after the last step.  T receives the
    # same A_i / B_i in the same order as the reference's per-step pushes (:185, :193).
    # Speculation: before the host blocks at a check and solves the T band (dsbev, up to ~35 ms at
    # N = 896), it may enqueue further steps, so the GPU keeps working during the eigensolve.  The
    # check reads only steps <= i, and steps after an even i touch no block <= i (partial reorth
    # at even steps), so D, S and the Ritz vectors are unchanged; a converged run discards the
    # extra steps, which is the cost.  speculate="auto" (default) enqueues up to the next check
    # when the residual bounds of the previous two checks, extrapolated geometrically, put this
    # check at least 100x above the tolerance, and one step when they put it above the tolerance
    # (host.speculation_depth) — on several ranks agreed once per check together with the
    # convergence test (rank 0's decisions, below), so ranks issue the same steps.
    # True: as many steps as the eigensolve is expected to last (the previous one scaled by
    # (N/N_prev)^2.7, over the measured time per step; one rank only); an int: a fixed count (tests).
    last_i = min(steps_cap, math.ceil(kryl_sz / b))
    enq = 0
    # Several ranks: each rank solves the same T band on its own host, and every rank must
    # enqueue the same steps (their collectives pair up).  So the two decisions a check takes —
    # converged, and (auto) how far to speculate before the next check — are all-gathered once
    # per check (rbl_allgather_host) and rank 0's are taken by every rank: eigensolves that
    # differ in the last bit across ranks (BLAS threading) cannot split the ranks' step counts.
    multi = ctx.nranks > 1
    next_depth = 0                                 # agreed auto depth for the next check

    def enqueue(upto):
        nonlocal enq
        t0 = time.perf_counter()
        while enq < upto:
            enq += 1
            ctx.step_async(enq, enq >= 2 and enq % 2 == 0)   # :164-184
        info.enqueue_ms += (time.perf_counter() - t0) * 1e3

    first = 1                                      # first unfetched step
    i = 0
    last_eig = last_n = None
    step_ms = None
    t_prev, i_prev, eig_prev = time.perf_counter(), 0, 0.0
    while True:
        i += 1                                     # step 1: first loop, :149-161; then :162-194
        is_check = check and i >= 2 and i * b > k and i % 4 == 0
        is_last = not (i * b < kryl_sz and i < steps_cap)
        if not (is_check or is_last):
            continue
        enqueue(i)
        # (one rank only: the count comes from host timings, and every rank must issue the
        # same steps — their collectives pair up)
        # (speculate may also be a fixed count of extra steps per check: tests)
        spec_to = i
        if speculate is not False and is_check and not is_last and i % 2 == 0:
            if speculate == "auto":
                spec_to = i + (next_depth if multi else speculation_depth(info.resid, tol))
            elif speculate is True:
                if ctx.nranks == 1 and last_eig and step_ms:
                    spec_to = i + int(last_eig * (i * b / last_n) ** 2.7 // step_ms)
            else:
                spec_to = i + int(speculate)
            spec_to = min(last_i, i + 4, spec_to)
            if spec_to > i:
                info.spec_steps += spec_to - i
                enqueue(spec_to)
        t0 = time.perf_counter()
        fetched = ctx.fetch(first, i + 1)
        t1 = time.perf_counter()
        info.fetch_ms += (t1 - t0) * 1e3
        if i > i_prev and t1 - t_prev > eig_prev:  # GPU time per step since the last fetch
            step_ms = ((t1 - t_prev) - eig_prev) * 1e3 / (i - i_prev)
        t_prev, i_prev, eig_prev = t1, i, 0.0
        for j, (Aj, Bj, st) in zip(range(first, i + 1), fetched):
            _record(Aj, Bj, st)
            T.insert_A(Aj)                         # :185
            if j == i and is_check:
                t0 = time.perf_counter()
                D, S = eig_topk(T.view(), k)       # :187-188
                dt = time.perf_counter() - t0
                info.eig_ms += dt * 1e3
                eig_prev = dt
                last_eig, last_n = dt * 1e3, i * b
                res = residual_norms(Bj, S, b, k)
                info.resid.append(float(res.max()) if res.size else 0.0)
                conv = bool(np.all(res <= tol))            # :189 (check_convergence)
                if multi:
                    depth = speculation_depth(info.resid, tol) if speculate == "auto" else 0
                    agreed = ctx.allgather([int(conv), depth])[0]   # rank 0's decisions
                    conv, next_depth = bool(agreed[0]), int(agreed[1])
                if conv:
                    info.converged = True
                    info.spec_wasted += spec_to - i
                    break
            T.insert_B(Bj, j)                      # :193
        first = i + 1
        if info.converged or is_last:
            break
    info.iters = i
    info.nblocks = i                               # Q_1..Q_i (length(Q))
    D = D[::-1].copy()
    # each Ritz vector's sign: its coefficient column's largest entry positive (host.fix_signs;
    # the eigensolvers disagree on signs, the reference returns dsbev's)
    S = fix_signs(S[:, ::-1])
    info.status = _lib.RBL_OK if info.converged else _lib.RBL_WARN_NOT_CONVERGED
    V = None
    if ritz and S.size:
        t0 = time.perf_counter()
        V = ctx.ritz(S.shape[0] // b, min(k, S.shape[1]), S)   # RBL_gpu.jl:219
        info.ritz_ms = (time.perf_counter() - t0) * 1e3
    return D, V, info


def RBL_gpu(A, k: int, b: int, *, device: int = 0, kryl_sz: int = KRYL_SZ_GPU, omega=None,
            seed: int = 0, reorth_order: int = 0, return_info: bool = False, basis_bits: int = 64,
            device_blocks: int = 0):
    """Drop-in for ``RBL_gpu(A::SparseMatrixCSC{Float64}, k, b)`` (RBL_gpu.jl:205):
    returns (D, V) — D the k largest-|lambda| eigenvalues (descending |lambda|), V n x k.
    device_blocks: Krylov blocks kept in HBM (RBL_OPT_DEVICE_BLOCKS: 0 all, -1 what fits —
    the reference's gpu_buffer_size — or G >= 3; older blocks spill to pinned host memory)."""
    with Context(device) as ctx:
        ctx.set_matrix(A)
        ctx.set_option(_lib.RBL_OPT_REORTH_ORDER, reorth_order)
        ctx.set_option(_lib.RBL_OPT_DEVICE_BLOCKS, device_blocks)
        D, V, info = lanczos(ctx, k, b, kryl_sz=kryl_sz, omega=omega, seed=seed,
                             basis_bits=basis_bits)
    return (D, V, info) if return_info else (D, V)
