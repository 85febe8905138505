"""GPU: the wide-band SpMM path at the headline's size (n = 1e7, ~100 nnz/row, b = 32, k = 20) with
half-width 1024 — the bench's `c4w_wideband` sub-record, where the column-panel kernel (kernel 7,
spmm_panel.hip) runs every A·Q_i of RBL_gpu.jl:176.

No oracle fixture exists at this size (the oracle's run of C4a took 617-873 s offline); the path
is pinned by size-independent properties and by the plain gather kernel, whose per-row sums run
in the CSR's order:

  * SpMM (`rbl_apply`, kernel 7): sampled row windows (the first and last rows and 64 evenly
    spaced windows of 512 rows) against SciPy's product of the same CSR rows downloaded from the
    device, every element within 1e-13 * (|A| |X|); linearity A (X1 + 2 X2) = A X1 + 2 A X2;
  * RBL_gpu to convergence on kernel 7: residuals ||A v - lambda v|| / |lambda| < 1e-7 (A v from
    SciPy over all 1e9 nonzeros), Ritz vectors orthonormal (1e-9), Rayleigh quotients within
    1e-10 of lambda, D sorted by descending |lambda| (P11);
  * the same Omega through the plain gather kernel (kernel 1, RBL_OPT_SPMM_KERNEL): the same step
    count, every step's A_i / B_{i+1} within 1e-9 relative and the eigenvalues within 1e-10
    relative — the panel kernel's rotated per-row sum order (spmm_panel.hip) changes nothing
    beyond rounding at full size.

Host memory: ~12 GB for the CSR, ~5 GB of n x 32 blocks; device: one context (~135 GB)."""
import time

import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu

N, HALFWIDTH, SEED, B, K = 10_000_000, 1024, 20261015, 32, 20
DENSITY = round(99 / (2 * HALFWIDTH), 6)         # ~100 nonzeros per row, as bench.py's sweep
T0 = time.perf_counter()
SPMM_TOL = 1e-13
TRACE_TOL = 1e-9
EIG_TOL = 1e-10


@pytest.fixture(scope="module")
def wide():
    import rbl
    plant = np.array([100.0 * (2 * K + 1 - l) for l in range(1, 2 * K + 1)])
    ctx = rbl.Context(0)
    ctx.gen_hashwindow(N, HALFWIDTH, DENSITY, SEED, plant)
    n, r0, r1, nnz = ctx.matrix_info()
    assert (n, r0, r1) == (N, 0, N) and 0.99e9 < nnz < 1.01e9
    print(f"[wideband] generated {nnz} nonzeros {time.perf_counter() - T0:.1f} s", flush=True)
    rowptr, col, val = ctx.get_matrix_csr()
    A = sp.csr_matrix((val, col, rowptr.astype(np.int32)), shape=(N, N))
    print(f"[wideband] CSR on the host {time.perf_counter() - T0:.1f} s", flush=True)
    yield rbl, ctx, A
    ctx.close()


def _windows():
    starts = np.linspace(512, N - 1024, 64).astype(np.int64)
    return [(0, 512)] + [(int(s), int(s) + 512) for s in starts] + [(N - 517, N)]


def test_wideband_fullsize_spmm_rows_and_linearity(wide):
    rbl, ctx, A = wide
    assert ctx.spmm_kernel_for(B) == 7           # the column panels
    rng = np.random.default_rng(11)
    X1 = rng.standard_normal((N, B))
    Y1 = ctx.apply(X1)
    aX = np.abs(X1)
    for a, b in _windows():
        As = A[a:b]
        bound = (abs(As) @ aX) * SPMM_TOL + 1e-300
        err = np.abs(Y1[a:b] - As @ X1)
        assert np.all(err <= bound), (a, float(np.max(err / bound)))
    print(f"[wideband] sampled rows checked {time.perf_counter() - T0:.1f} s", flush=True)
    X2 = rng.standard_normal((N, B))
    Y2 = ctx.apply(X2)
    X1 += 2.0 * X2
    Y3 = ctx.apply(X1)
    Y1 += 2.0 * Y2
    aX = np.abs(X1)
    aX += 4.0 * np.abs(X2)
    for a, b in _windows():
        bound = 3 * SPMM_TOL * (abs(A[a:b]) @ aX)
        assert np.all(np.abs(Y3[a:b] - Y1[a:b]) <= bound + 1e-300), a


def test_wideband_fullsize_rbl_gpu_panels_vs_gather(wide):
    rbl, ctx, A = wide
    omega = np.random.default_rng(SEED + 5).standard_normal((N, B))
    ctx.set_option(2, 0)                          # automatic: the column panels
    assert ctx.spmm_kernel_for(B) == 7
    D, V, info = rbl.lanczos(ctx, K, B, omega=omega, trace=True)
    print(f"[wideband] panels: {info.iters} steps {time.perf_counter() - T0:.1f} s", flush=True)
    assert info.converged and D.shape == (K,) and V.shape == (N, K)
    assert 3900 < D[0] < 4100                     # the planted top (100 (2k+1-l), perturbed)
    assert np.all(np.diff(np.abs(D)) <= 0)
    AV = A @ V
    res = np.linalg.norm(AV - V * D, axis=0) / np.abs(D)
    assert res.max() < 1e-7, res
    G = V.T @ V
    assert np.abs(G - np.eye(K)).max() < 1e-9
    rq = np.einsum("ij,ij->j", V, AV) / np.einsum("ij,ij->j", V, V)
    assert np.all(np.abs(rq - D) <= 1e-10 * np.abs(D))
    del V, AV
    ctx.set_option(2, 1)                          # the plain gather: CSR-order row sums
    try:
        assert ctx.spmm_kernel_for(B) == 1
        Dg, _, infog = rbl.lanczos(ctx, K, B, omega=omega, trace=True, ritz=False)
    finally:
        ctx.set_option(2, 0)
    print(f"[wideband] gather: {infog.iters} steps {time.perf_counter() - T0:.1f} s", flush=True)
    assert infog.converged and infog.iters == info.iters
    for i in range(info.iters):
        for x, y in ((info.trace_A[i], infog.trace_A[i]), (info.trace_B[i], infog.trace_B[i])):
            assert np.abs(x - y).max() <= TRACE_TOL * np.abs(y).max(), i
    rel = np.abs(Dg - D) / np.abs(D)
    assert rel.max() < EIG_TOL, rel
