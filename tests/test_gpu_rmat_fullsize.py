"""GPU: BASELINE config 4 at full size (C4b: R-MAT scale 24, n = 1e7, ~1e9 nonzeros, b = 32,
k = 20 — the bench's `c4b_rmat` workload, as drawn).

Against the oracle at full size: tests/golden/make_fullsize.py c4b_full ran the oracle on this
very matrix offline in the build container (the R-MAT CSR built in chunks, bit-exact with
matgen.rmat_csr; block CGS evaluated block by block) and committed golden_c4b_full.npz;
test_c4b_full_size_vs_oracle feeds the fixture's Omega and checks the step count, the
eigenvalues (< 1e-10 relative) and each Ritz vector's 16 largest entries (1e-6, up to sign).

Beside it, size-independent properties:

  * SpMM (`rbl_apply`: the segmented gather + long-row fixup the bench runs) on sampled rows
    against SciPy's product of the same CSR rows downloaded from the device: the 64 highest-
    degree rows (hubs of up to ~1e6 nonzeros, cut into 4,096-nonzero segments whose partial rows
    k_seg_fixup sums), 32 windows of 256 rows spread over [0, n) (packed short-row tasks), and
    the last rows; every element within 1e-13 * (|A| |X|) (the kernel only reorders the fp64
    sums; same bound as test_gpu_spmm);
  * linearity of the SpMM: A (X1 + 2 X2) = A X1 + 2 A X2 within 3x that bound;
  * RBL_gpu to convergence (RBL_gpu.jl:134-219 semantics): every Ritz pair's residual
    ||A v - lambda v|| / |lambda| < 1e-7 (A v by SciPy over all 1e9 nonzeros), Ritz vectors
    orthonormal (|V^T V - I| < 1e-9), Rayleigh quotients equal to lambda within 1e-10
    relative, D sorted by descending |lambda| (P11).

Host memory: ~12 GB for the downloaded CSR, ~8 GB of n x 32 blocks; device: the context's
~125 GB (basis of 39 fp64 blocks + matrix)."""
import time

import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu

N, SCALE, EDGES, SEED, B, K = 10_000_000, 24, 660_000_000, 20261015, 32, 20
T0 = time.perf_counter()
SPMM_TOL = 1e-13
RES_TOL = 1e-7
ORTH_TOL = 1e-9
RAYLEIGH_TOL = 1e-10
SEG_LEN = 4096          # kernels.hpp kSegLen: nonzeros per long-row segment


def _log(msg):
    print(f"[c4b fullsize] {msg} {time.perf_counter() - T0:.1f} s", flush=True)


@pytest.fixture(scope="module")
def full():
    """One context with the bench's C4b matrix generated on the device, and its CSR on the host."""
    import rbl
    plant = np.array([100.0 * (2 * K + 1 - l) for l in range(1, 2 * K + 1)])
    ctx = rbl.Context(0)
    ctx.gen_rmat(N, SCALE, EDGES, SEED, plant)
    n, r0, r1, nnz = ctx.matrix_info()
    assert (n, r0, r1) == (N, 0, N) and 0.95e9 < nnz < 1.05e9
    _log(f"generated {nnz} nonzeros")
    rowptr, col, val = ctx.get_matrix_csr()
    _log("CSR downloaded")
    A = sp.csr_matrix((val, col, rowptr.astype(np.int32)), shape=(N, N))
    yield rbl, ctx, A
    ctx.close()


def _row_sets(A):
    deg = np.diff(A.indptr)
    hubs = np.sort(np.argsort(-deg)[:64])
    assert deg[hubs].max() > 100 * SEG_LEN        # the top hub spans > 100 segments
    assert (deg[hubs] > SEG_LEN).sum() >= 32      # and most sampled hubs are segmented
    starts = np.linspace(1024, N - 2048, 32).astype(np.int64)
    return [hubs] + [np.arange(s, s + 256) for s in starts] + [np.arange(N - 300, N)]


def test_c4b_fullsize_spmm_sampled_rows_and_linearity(full):
    rbl, ctx, A = full
    assert ctx.spmm_kernel_for(B) == 6            # the segmented gather of the bench line
    rows = _row_sets(A)
    rng = np.random.default_rng(7)
    X1 = rng.standard_normal((N, B))
    Y1 = ctx.apply(X1)
    _log("A X1")
    aX = np.abs(X1)
    for r in rows:
        As = A[r]
        ref = As @ X1
        bound = (abs(As) @ aX) * SPMM_TOL + 1e-300
        err = np.abs(Y1[r] - ref)
        assert np.all(err <= bound), (int(r[0]), float(np.max(err / bound)))
    _log("sampled rows checked")
    X2 = rng.standard_normal((N, B))
    Y2 = ctx.apply(X2)
    X1 += 2.0 * X2
    Y3 = ctx.apply(X1)
    Y1 += 2.0 * Y2
    aX = np.abs(X1)
    aX += 4.0 * np.abs(X2)
    for r in rows:
        bound = 3 * SPMM_TOL * (abs(A[r]) @ aX)
        assert np.all(np.abs(Y3[r] - Y1[r]) <= bound + 1e-300), int(r[0])
    _log("linearity checked")


def test_c4b_fullsize_rbl_gpu(full):
    rbl, ctx, A = full
    D, V, info = rbl.lanczos(ctx, K, B, seed=SEED + 2, check=True, ritz=True)
    _log(f"RBL_gpu: {info.iters} steps")
    assert info.converged and D.shape == (K,) and V.shape == (N, K)
    assert np.all(np.diff(np.abs(D)) <= 0)                        # P11
    AV = A @ V
    _log("A V on the host")
    res = np.linalg.norm(AV - V * D, axis=0) / np.abs(D)
    assert res.max() < RES_TOL, res
    G = V.T @ V
    assert np.abs(G - np.eye(K)).max() < ORTH_TOL, np.abs(G - np.eye(K)).max()
    rq = np.einsum("ij,ij->j", V, AV) / np.einsum("ij,ij->j", V, V)
    assert np.all(np.abs(rq - D) <= RAYLEIGH_TOL * np.abs(D)), np.abs(rq - D) / np.abs(D)


def test_c4b_full_size_vs_oracle(full):
    """BASELINE config 4 against the oracle's own run at n = 1e7 (golden_c4b_full.npz): the
    device-generated R-MAT matrix (relabel off: the matrix as drawn) is the fixture's (same
    nonzero count; the generator is bit-exact, test_gpu_rmat), the fixture's Omega, the same
    number of block steps to convergence, eigenvalues within 1e-10 relative, Ritz vectors'
    largest entries within 1e-6 up to sign."""
    import os
    rbl, ctx, A = full
    g = np.load(os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden", "golden_c4b_full.npz"))
    cfg = {k[4:]: g[k].item() for k in g.files if k.startswith("cfg_")}
    assert (cfg["n"], cfg["scale"], cfg["edges"], cfg["seed"], cfg["b"], cfg["k"]) == (N, SCALE, EDGES, SEED, B, K)
    assert A.nnz == int(g["nnz"])
    omega = np.random.default_rng(cfg["omega_seed"]).standard_normal((N, B))
    D, V, info = rbl.lanczos(ctx, K, B, omega=omega, trace=True)
    del omega
    _log(f"vs oracle: {info.iters} steps")
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
