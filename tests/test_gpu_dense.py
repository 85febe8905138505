"""GPU parity of the dense-A path — RBL_gpu(A::Matrix{Float64}, k, b) (RBL_gpu.jl:205;
images.jl:20-33 runs RBL on a dense B^T B) — against the oracle on the same inputs.

A * Q runs as a panel GEMM on fp64 MFMA (rbl_set_matrix_dense).  Tolerances as the sparse
path (test_gpu_parity.py): eigenvalues 1e-10 relative, Ritz residual 1e-7, rbl_apply 1e-12.
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import rbl_oracle as o

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rbl():
    import rbl as _r
    return _r


def dense_planted(n, k, seed=5):
    """Dense symmetric: small random symmetric part + planted top spectrum (orthogonal frame)."""
    rng = np.random.default_rng(seed)
    G = rng.standard_normal((n, n)) / np.sqrt(n)
    A = (G + G.T) * 0.5
    Qf, _ = np.linalg.qr(rng.standard_normal((n, 2 * k)))
    lam = 100.0 * (2 * k + 1 - np.arange(1, 2 * k + 1))
    return A + (Qf * lam) @ Qf.T


@pytest.mark.parametrize("n,b", [(1000, 1), (999, 5), (1000, 8), (2048, 16), (3001, 32)])
def test_dense_apply(rbl, n, b):
    A = dense_planted(n, 5)
    X = np.random.default_rng(1).standard_normal((n, b))
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        assert ctx.spmm_kernel_for(b) == 4
        Y = ctx.apply(X)
        with pytest.raises(rbl.RBLError):
            ctx.get_matrix_csr()
    ref = A @ X
    assert np.abs(Y - ref).max() <= 1e-12 * np.abs(ref).max()


@pytest.mark.parametrize("n,b", [(1500, 8), (3001, 16), (2048, 32)])
def test_dense_eigenpairs(rbl, n, b):
    k = 10
    A = dense_planted(n, k)
    omega = np.random.default_rng(7).standard_normal((n, b))
    ref = o.RBL_gpu_semantics(A, k, b, omega=omega, qr_mode="posdiag", reorth_mode="cgs")
    D, V, info = rbl.RBL_gpu(A, k, b, omega=omega, return_info=True)
    assert ref.converged and info.converged
    assert np.all(np.abs(D - ref.D) <= 1e-10 * np.abs(ref.D))
    res = np.linalg.norm(A @ V - V * D[None, :], axis=0) / np.abs(D)
    assert res.max() < 1e-7
    # the same matrix through the sparse path gives the same spectrum
    D2, _ = rbl.RBL_gpu(sp.csr_matrix(A), k, b, omega=omega)
    assert np.all(np.abs(D - D2) <= 1e-10 * np.abs(D2))


def test_dense_multirank(rbl):
    from test_gpu_multirank import run_ranks
    k, b, n = 10, 16, 2500
    A = dense_planted(n, k)
    omega = np.random.default_rng(3).standard_normal((n, b))
    D1, V1 = rbl.RBL_gpu(A, k, b, omega=omega)

    def fn(ctx, r):
        ctx.set_matrix(A)
        _, r0, r1, _ = ctx.matrix_info()
        return rbl.lanczos(ctx, k, b, omega=omega[r0:r1])

    parts = run_ranks(rbl, 3, fn)
    for D, _, info in parts:
        assert info.converged
        assert np.all(np.abs(D - D1) <= 1e-10 * np.abs(D1))
    V = np.vstack([p[1] for p in parts])
    assert np.all(1 - np.abs(np.sum(V * V1, axis=0)) < 1e-8)
