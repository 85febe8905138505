"""world_size = 2 (and 3) gloo tests of the row-partitioned path on CPU.

Each rank plans its rows and halos with librbl_hip.so's host planning entry points and runs
the library's distributed step order (tests/dist_emul.py) with gloo standing in for RCCL:
  * the halo-exchanged SpMM reproduces A @ X row for row;
  * the per-step A_i / B_i of the partitioned run match the single-process oracle
    (block-CGS partial reorth, positive-diagonal QR) within 1e-10 relative, on an
    nnz-balanced split of a random sparse matrix and on the row-sliced hash-window generator;
  * every rank ends with the same T_j entries (the host eigensolve sees identical input);
  * on an R-MAT pattern, the push/pull split of the indexed halo (dist_emul.PushPullRows):
    the same SpMM and traces, with fewer rows moved than pulling every referenced row.
The device-side transport of the same code path is exercised on the GPU box by
tests/test_gpu_multirank.py.
"""
import os
import socket

import numpy as np
import pytest
import scipy.sparse as sp

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rand_sym(n, density, seed):
    R = sp.random(n, n, density=density, random_state=seed, format="csr")
    A = sp.csr_matrix(R + R.T + sp.diags(np.linspace(50.0, 1.0, n)))
    A.sort_indices()
    return A


def _worker(rank, world, port, case):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _run_case(case)
    finally:
        dist.destroy_process_group()


def _run_case(case):
    import dist_emul as de
    from oracle import matgen
    from oracle import rbl_oracle as o

    b, steps = 8, 8
    if case == "csc":
        A = _rand_sym(1500, 0.004, 5)
        M = de.DistRows(A.shape[0], csr_global=A)
    elif case == "rmat_push":   # power-law pattern, the push/pull split of the indexed halo
        A = matgen.rmat_csr(3000, 12, 60_000, 7, matgen.planted_spectrum(6))
        M = de.PushPullRows(A.shape[0], csr_global=A)
        assert M.symmetric
        moved = int(de.allreduce(np.array([float(M.rows_moved)]))[0])
        r0, r1 = M.r0, M.r1
        offr = A[r0:r1].tocoo()
        pull_all = np.unique(offr.col[(offr.col < r0) | (offr.col >= r1)]).size
        pull_all = int(de.allreduce(np.array([float(pull_all)]))[0])
        assert 0 < moved < pull_all, (moved, pull_all)   # the hubs' rows stay home
    else:
        n, W, p, seed = 2400, 30, 0.6, 17
        plant = matgen.planted_spectrum(6)
        A = matgen.hashwindow_csr(n, W, p, seed, plant)
        M = de.DistRows(n, hashwindow=(W, p, seed, plant))
    n = A.shape[0]
    me, P = dist.get_rank(), dist.get_world_size()
    # the slices tile [0, n) and every rank agrees on them
    bounds = de.allgather_i64(M.bounds)
    assert np.all(bounds == bounds[0]) and bounds[0][0] == 0 and bounds[0][-1] == n
    # halo-exchanged SpMM == A @ X on my rows
    X = np.random.default_rng(1).standard_normal((n, b))
    Y = M.spmm(X[M.r0:M.r1])
    ref = A[M.r0:M.r1] @ X
    assert np.abs(Y - ref).max() <= 1e-12 * max(1.0, np.abs(ref).max())
    # the partitioned Lanczos trace == the single-process oracle trace
    omega = np.random.default_rng(2).standard_normal((n, b))
    tA, tB, _ = de.dist_lanczos_trace(M, omega[M.r0:M.r1].copy(), steps)
    res = o.RBL_gpu_semantics(A, 4, b, omega=omega, qr_mode="posdiag", reorth_mode="cgs",
                              check=False, max_steps=steps, trace=True)
    for a, a_ref in zip(tA, res.trace["A"]):
        assert np.abs(a - a_ref).max() <= 1e-10 * np.abs(a_ref).max()
    for bb, b_ref in zip(tB, res.trace["B"]):
        assert np.abs(bb - b_ref).max() <= 1e-10 * np.abs(b_ref).max()
    # identical T_j input on every rank
    allA = de.allgather_i64(np.frombuffer(np.stack(tA).tobytes(), dtype=np.int64))
    assert np.all(allA == allA[0])


@pytest.mark.parametrize("world,case", [(2, "csc"), (2, "hashwindow"), (3, "csc"),
                                        (2, "rmat_push"), (3, "rmat_push")])
def test_gloo_partitioned_lanczos(world, case):
    mp.spawn(_worker, args=(world, _free_port(), case), nprocs=world, join=True)
