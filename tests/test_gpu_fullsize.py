"""GPU: BASELINE's headline configuration at full size (C4a: n = 1e7, ~100 nnz/row, b = 32,
k = 20 — the bench workload).

Against the oracle at full size: tests/golden/make_fullsize.py ran the oracle (the CPU
restatement of RBL.jl with the GPU driver's bounds) on this very matrix offline, in the build
container (873 s, 44.7 GB peak RSS, block CGS evaluated block by block), and committed
golden_c4a.npz (round 6: regenerated with the per-step traces, 617 s; D unchanged).
test_c4a_full_size_vs_oracle feeds the fixture's Omega and checks the step count, every
step's A_i and B_{i+1} (relative 1e-8), the eigenvalues (< 1e-10 relative) and each Ritz
vector's 16 largest entries (1e-6, up to sign).

Beside it, size-independent properties:

  * SpMM (`rbl_apply`, the band-tile kernel the bench runs): sampled row windows — the first and
    last rows (ragged last tile), and 64 evenly spaced windows of 512 rows — against SciPy's
    product of the same CSR rows downloaded from the device; every element within
    1e-13 * (|A| |X|) (the kernel only reorders the fp64 sums; same bound as test_gpu_spmm);
  * linearity of the SpMM: A (X1 + 2 X2) = A X1 + 2 A X2 within the same bound;
  * RBL_gpu to convergence (RBL_gpu.jl:134-219 semantics): every Ritz pair's residual
    ||A v - lambda v|| / |lambda| < 1e-7 (A v from SciPy over all 1e9 nonzeros), Ritz vectors
    orthonormal (|V^T V - I| < 1e-9), Rayleigh quotients v^T A v equal to lambda within 1e-10
    relative, D sorted by descending |lambda| (P11);
  * the mixed mode (fp32 basis, config 5's arithmetic) on the same matrix: eigenvalues within
    1e-6 relative of the fp64 run and residuals < 1e-5 (the tolerances of
    test_gpu_fp32_basis.py).

Host memory: ~12 GB for the downloaded CSR, ~4 GB of n x 32 blocks; device: the context's
~125 GB (basis of 39 fp64 blocks + matrix)."""
import time

import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu

N, HALFWIDTH, DENSITY, SEED, B, K = 10_000_000, 64, 0.7734, 20261015, 32, 20
T0 = time.perf_counter()
SPMM_TOL = 1e-13
RES_TOL = 1e-7
ORTH_TOL = 1e-9
RAYLEIGH_TOL = 1e-10
EIG_TOL_MIXED = 1e-6
RES_TOL_MIXED = 1e-5


@pytest.fixture(scope="module")
def full():
    """One context with the bench's C4a matrix generated on the device, and its CSR on the host."""
    import rbl
    plant = np.array([100.0 * (2 * K + 1 - l) for l in range(1, 2 * K + 1)])
    ctx = rbl.Context(0)
    ctx.gen_hashwindow(N, HALFWIDTH, DENSITY, SEED, plant)
    n, r0, r1, nnz = ctx.matrix_info()
    assert (n, r0, r1) == (N, 0, N) and 0.99e9 < nnz < 1.01e9
    print(f"[fullsize] generated {nnz} nonzeros {time.perf_counter() - T0:.1f} s", flush=True)
    rowptr, col, val = ctx.get_matrix_csr()
    print(f"[fullsize] CSR downloaded {time.perf_counter() - T0:.1f} s", flush=True)
    # nnz < 2^31: int32 indices keep SciPy from widening 4 GB of column indices
    A = sp.csr_matrix((val, col, rowptr.astype(np.int32)), shape=(N, N))
    yield rbl, ctx, A
    ctx.close()


def _windows():
    starts = np.linspace(512, N - 1024, 64).astype(np.int64)
    return [(0, 512)] + [(int(s), int(s) + 512) for s in starts] + [(N - 517, N)]


def _check_rows(A, Y, X):
    aX = np.abs(X)                               # once: 2.56 GB, not per window
    for a, b in _windows():
        As = A[a:b]
        ref = As @ X
        bound = (abs(As) @ aX) * SPMM_TOL + 1e-300
        err = np.abs(Y[a:b] - ref)
        assert np.all(err <= bound), (a, float(np.max(err / bound)))


def test_fullsize_spmm_sampled_rows_and_linearity(full):
    rbl, ctx, A = full
    print(f"[fullsize] matrix ready {time.perf_counter() - T0:.1f} s", flush=True)
    assert ctx.spmm_kernel_for(B) == 5           # the band-tile kernel of the bench line
    rng = np.random.default_rng(7)
    X1 = rng.standard_normal((N, B))             # C order: SciPy copies F-order operands per product
    Y1 = ctx.apply(X1)
    print(f"[fullsize] A X1 {time.perf_counter() - T0:.1f} s", flush=True)
    _check_rows(A, Y1, X1)
    print(f"[fullsize] sampled rows checked {time.perf_counter() - T0:.1f} s", flush=True)
    X2 = rng.standard_normal((N, B))
    Y2 = ctx.apply(X2)
    X1 += 2.0 * X2                               # X3 = X1 + 2 X2 (in place: host memory)
    Y3 = ctx.apply(X1)
    Y1 += 2.0 * Y2
    # each side is within SPMM_TOL |A| (|X1| + 2 |X2|) <= SPMM_TOL |A| (|X3| + 4 |X2|) of
    # A X3 (plus the rounding of X3 itself): 3x that bounds the difference
    aX = np.abs(X1)
    aX += 4.0 * np.abs(X2)
    for a, b in _windows():
        bound = 3 * SPMM_TOL * (abs(A[a:b]) @ aX)
        assert np.all(np.abs(Y3[a:b] - Y1[a:b]) <= bound + 1e-300), a


def _check_pairs(A, D, V, res_tol, orth_tol, rayleigh_tol):
    assert np.all(np.diff(np.abs(D)) <= 0)                        # P11: descending |lambda|
    AV = A @ V
    print(f"[fullsize] A V on the host {time.perf_counter() - T0:.1f} s", flush=True)
    res = np.linalg.norm(AV - V * D, axis=0) / np.abs(D)
    assert res.max() < res_tol, res
    G = V.T @ V
    assert np.abs(G - np.eye(V.shape[1])).max() < orth_tol, np.abs(G - np.eye(V.shape[1])).max()
    rq = np.einsum("ij,ij->j", V, AV) / np.einsum("ij,ij->j", V, V)
    assert np.all(np.abs(rq - D) <= rayleigh_tol * np.abs(D)), np.abs(rq - D) / np.abs(D)
    return res


def test_c4a_full_size_vs_oracle(full):
    """BASELINE's headline config against the oracle's own run at n = 1e7 (golden_c4a.npz): the
    device-generated matrix is the fixture's (same nonzero count; the generator is bit-exact,
    test_gpu_parity), the fixture's Omega, the same number of block steps to convergence,
    eigenvalues within 1e-10 relative, Ritz vectors' largest entries within 1e-6 up to sign."""
    import os
    rbl, ctx, A = full
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_c4a.npz"))
    cfg = {k[4:]: g[k].item() for k in g.files if k.startswith("cfg_")}
    assert (cfg["n"], cfg["halfwidth"], cfg["density"], cfg["seed"], cfg["b"], cfg["k"]) == \
        (N, HALFWIDTH, DENSITY, SEED, B, K)
    assert A.nnz == int(g["nnz"])
    omega = np.random.default_rng(cfg["omega_seed"]).standard_normal((N, B))
    D, V, info = rbl.lanczos(ctx, K, B, omega=omega, trace=True)
    del omega
    print(f"[fullsize] vs oracle: {info.iters} steps {time.perf_counter() - T0:.1f} s", flush=True)
    assert info.converged and info.iters == int(g["iters"])
    # the block-step semantics at full size (RBL_gpu.jl:153-161, 176-184): every step's A_i and
    # B_{i+1} against the oracle's, relative 1e-8 of the block's largest entry (as the small-n
    # trace tests); positive-diagonal R on both sides, so no sign normalisation
    tA, tB = g["trace_A"], g["trace_B"]
    assert len(info.trace_A) == len(info.trace_B) == tA.shape[0] == tB.shape[0] == info.iters
    for i in range(info.iters):
        da = np.abs(info.trace_A[i] - tA[i]).max() / np.abs(tA[i]).max()
        db = np.abs(info.trace_B[i] - tB[i]).max() / np.abs(tB[i]).max()
        assert da < 1e-8 and db < 1e-8, (i, da, db)
    rel = np.abs(D - g["D"]) / np.abs(g["D"])
    assert rel.max() < 1e-10, rel
    idx, val = g["top_idx"], g["top_val"]
    for j in range(K):
        v = V[idx[:, j], j]
        s = np.sign(v @ val[:, j])
        assert np.abs(s * v - val[:, j]).max() < 1e-6, (j, np.abs(s * v - val[:, j]).max())


def test_fullsize_rbl_gpu_fp64_and_mixed(full):
    rbl, ctx, A = full
    D, V, info = rbl.lanczos(ctx, K, B, seed=SEED + 2, check=True, ritz=True)
    print(f"[fullsize] fp64 RBL_gpu: {info.iters} steps {time.perf_counter() - T0:.1f} s", flush=True)
    assert info.converged and D.shape == (K,) and V.shape == (N, K)
    # the planted spectrum (100 (2k+1-l), perturbed by the N(0,1) band) dominates the top
    assert 3900 < D[0] < 4100
    _check_pairs(A, D, V, RES_TOL, ORTH_TOL, RAYLEIGH_TOL)
    del V
    D32, V32, info32 = rbl.lanczos(ctx, K, B, seed=SEED + 2, check=True, ritz=True, basis_bits=32)
    print(f"[fullsize] mixed RBL_gpu: {info32.iters} steps {time.perf_counter() - T0:.1f} s", flush=True)
    assert info32.converged
    assert np.all(np.abs(D32 - D) <= EIG_TOL_MIXED * np.abs(D)), np.abs(D32 - D) / np.abs(D)
    res = np.linalg.norm(A @ V32 - V32 * D32, axis=0) / np.abs(D32)
    assert res.max() < RES_TOL_MIXED, res
