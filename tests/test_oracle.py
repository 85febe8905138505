"""CPU: pin the oracle against the reference's own known-answer suites and check its helpers.

Julia/Unit Testing/test.jl:16-50 with mod_dec.jl / slow_dec.jl / step_dec.jl:3-7 —
norm of the relative eigenvalue error < 1e-13 for k = 5, b = 5.
"""
import numpy as np
import pytest

from oracle import matgen
from oracle import rbl_oracle as o


@pytest.mark.parametrize("suite", ["moderate", "slow", "step"])
def test_known_answer_suites(suite):
    gen, ns, k, b = o.KNOWN_ANSWER_SUITES[suite]
    for n in ns:
        A, eig = gen(n, k)
        r = o.RBL(A, k, b, seed=1000 + n)
        assert r.converged
        err = np.linalg.norm((r.D - eig) / eig)
        assert err < o.KNOWN_ANSWER_TOL, (suite, n, err)


def test_insert_band_matches_dense_T():
    rng = np.random.default_rng(0)
    b, m = 3, 4
    As = [rng.standard_normal((b, b)) for _ in range(m)]
    As = [a + a.T for a in As]
    Bs = [np.triu(rng.standard_normal((b, b))) for _ in range(m)]
    T = o.insertA(As[0], b)
    o.insertB(Bs[0], T, b, 1)
    for i in range(1, m):
        T = np.hstack([T, o.insertA(As[i], b)])
        if i < m - 1:
            o.insertB(Bs[i], T, b, i + 1)
    N = m * b
    dense = np.zeros((N, N))
    for i in range(m):
        dense[i * b:(i + 1) * b, i * b:(i + 1) * b] = As[i]
        if i < m - 1:
            dense[(i + 1) * b:(i + 2) * b, i * b:(i + 1) * b] = Bs[i]
            dense[i * b:(i + 1) * b, (i + 1) * b:(i + 2) * b] = Bs[i].T
    w, _ = o.dsbev(T)
    assert np.allclose(np.sort(w), np.linalg.eigvalsh(dense), atol=1e-12)


def test_sort_eig_abs_stable_and_magnitude():
    D = np.array([-5.0, 1.0, 5.0, -2.0, 3.0])
    V = np.eye(5)
    d, v = o.sort_eig_abs(D, V, 3)
    assert list(d) == [3.0, -5.0, 5.0]      # stable: -5 (index 0) before 5 (index 2)
    assert v.shape == (5, 3)


def test_mgs_and_cgs_reorth_agree():
    rng = np.random.default_rng(1)
    n, b = 200, 4
    # orthonormal earlier blocks (as in Lanczos) + targets with a small loss of orthogonality
    Qa = np.linalg.qr(rng.standard_normal((n, 5 * b)))[0]
    Q = [Qa[:, j * b:(j + 1) * b].copy() for j in range(5)]
    for t in (3, 4):
        Q[t] += 1e-6 * (Q[0] @ rng.standard_normal((b, b)) + Q[1] @ rng.standard_normal((b, b)))
    Q1 = [q.copy() for q in Q]
    Q2 = [q.copy() for q in Q]
    o.part_reorth(Q1, "mgs")
    o.part_reorth(Q2, "cgs")
    for a, c in zip(Q1, Q2):
        assert np.allclose(a, c, atol=1e-12)


def test_nonconvergence_is_reported():
    A, _ = o.slow_decay_matrix(2000, 5)
    r = o.RBL(A, 5, 5, seed=3, kryl_sz=60)
    assert not r.converged
    assert r.V.shape[0] == 2000


def test_posdiag_qr_gives_same_eigenvalues():
    A, eig = o.moderate_decay_matrix(300, 5)
    r1 = o.RBL(A, 5, 5, seed=11, qr_mode="householder")
    r2 = o.RBL(A, 5, 5, seed=11, qr_mode="posdiag")
    assert np.allclose(r1.D, r2.D, rtol=1e-13)


def test_mixed_mode_oracle_tracks_fp64():
    """RBL_gpu_mixed (FLOAT = Float32 GPU semantics) against the fp64 restatement on
    a planted-spectrum matrix: the fp32 basis moves converged eigenvalues by ~1e-9 relative
    here; the bound asserted is 1e-6 (the GPU fp32-basis parity tests use the same bound)."""
    from oracle import matgen
    k, b = 10, 16
    A = matgen.hashwindow_csr(3000, 64, 0.3, 5, matgen.planted_spectrum(k))
    omega = np.random.default_rng(2).standard_normal((A.shape[0], b))
    r64 = o.RBL_gpu_semantics(A, k, b, omega=omega, qr_mode="posdiag")
    r32 = o.RBL_gpu_mixed(A, k, b, omega=omega)
    assert r64.converged and r32.converged
    assert np.max(np.abs(r32.D - r64.D) / np.abs(r64.D)) < 1e-6
    res = np.linalg.norm(A @ r32.V - r32.V * r32.D[None, :], axis=0) / np.abs(r32.D)
    assert res.max() < 1e-5


def test_rmat_restatement_properties():
    """R-MAT oracle (C4b): symmetric, sorted, every diagonal present with the planted spectrum,
    power-law skew (the top 1 % of rows hold far more than 1 % of the nonzeros), and row
    slices equal to the rows of the full matrix."""
    n, k = 4000, 5
    plant = matgen.planted_spectrum(k)
    A = matgen.rmat_csr(n, 12, 60_000, 11, plant)
    assert abs(A - A.T).max() == 0
    assert np.all(A.diagonal() != 0)
    stride = n // len(plant)
    d = A.diagonal()
    assert np.all(np.abs(d[::stride][:len(plant)] - plant) <= 1.0)
    deg = np.diff(A.indptr)
    top = np.sort(deg)[::-1][: n // 100].sum()
    assert top > 0.1 * A.nnz
    part = matgen.rmat_csr(n, 12, 60_000, 11, plant, row_begin=1000, row_end=2500)
    assert (part != A[1000:2500]).nnz == 0


def test_rmat_relabel_is_a_symmetric_permutation():
    """RBL_OPT_RELABEL's restatement: matgen.rmat_csr(relabel=True) is P A P^T for the seeded
    Feistel permutation rmat_relabel (so the spectrum is A's), row slices tile it, and the
    permutation and its inverse are bijections of [0, n)."""
    import scipy.sparse as sp
    from oracle import matgen as m
    n, seed = 3000, 5
    A = m.rmat_csr(n, 12, n * 30, seed, m.planted_spectrum(5))
    B = m.rmat_csr(n, 12, n * 30, seed, m.planted_spectrum(5), relabel=True)
    perm = m.rmat_relabel(n, seed, np.arange(n))
    assert np.array_equal(np.sort(perm), np.arange(n))
    assert np.array_equal(m.rmat_relabel(n, seed, perm, inverse=True), np.arange(n))
    P = sp.csr_matrix((np.ones(n), (perm, np.arange(n))), shape=(n, n))
    assert abs(P @ A @ P.T - B).max() == 0.0 and abs(B - B.T).max() == 0.0
    part = m.rmat_csr(n, 12, n * 30, seed, m.planted_spectrum(5), relabel=True, row_begin=700,
                      row_end=1900)
    assert abs(part - B[700:1900]).max() == 0.0
    # the hubs (R-MAT's low ids) no longer sit in the first rows
    deg = np.diff(B.indptr)
    assert deg[: n // 8].sum() < 0.3 * deg.sum() < np.diff(A.indptr)[: n // 8].sum()


def test_mixed_mode_step_suite_spurious_pairs():
    """Documents a property of the reference's mixed mode (FLOAT = Float32, README.md:69) on its
    own step suite (test.jl:40-50, n = 1e5): the T-based convergence test (common.jl:56-65)
    passes while the returned top-k holds spurious values beside the true 10n, 9n, 8n — the
    fp32 basis loses orthogonality against eigenvectors 1e5 times the bulk.  The fp64 oracle
    meets the suite's 1e-13 on the same Omega."""
    n = 100_000
    A, eig = o.step_decay_matrix(n, 5)
    om = np.random.default_rng(1).standard_normal((n, 5))
    r32 = o.RBL_gpu_mixed(A, 5, 5, omega=om)
    r64 = o.RBL_gpu_semantics(A, 5, 5, omega=om, qr_mode="posdiag", reorth_mode="cgs")
    assert r32.converged and r64.converged
    assert np.linalg.norm((r64.D - eig) / eig) < o.KNOWN_ANSWER_TOL
    assert np.linalg.norm((r32.D - eig) / eig) > 1e-2           # spurious values in the top 5
    assert abs(r32.D[0] - eig[0]) < 1e-6 * eig[0]                # the top one is right
    res = np.linalg.norm(A @ r32.V - r32.V * r32.D, axis=0) / np.abs(r32.D)
    assert res.max() > 1e-5                                      # ... and not eigenpairs of A


def test_hashwindow_chunked_is_the_same_matrix():
    """matgen.hashwindow_csr_chunked (the form the full-size fixtures and bench --cpu-fixed-n use)
    builds hashwindow_csr's matrix bit for bit, chunk boundaries anywhere."""
    plant = matgen.planted_spectrum(20)
    A = matgen.hashwindow_csr(30000, 64, 0.7734, 11, plant)
    for chunk in (997, 30000, 4096):
        B = matgen.hashwindow_csr_chunked(30000, 64, 0.7734, 11, plant, chunk)
        assert np.array_equal(A.indptr, B.indptr) and np.array_equal(A.indices, B.indices)
        assert np.array_equal(A.data, B.data)


def test_c1_random_symmetric_as_defined():
    """SURVEY §8(d) C1 as defined (A = R + R^T, 1 % density, N(0,1), planted diagonal): symmetric,
    seeded (the same matrix twice), and the oracle's top k = 10 at b = 8 are the planted values to
    the random part's perturbation, converged with small residuals."""
    k = 10
    plant = matgen.planted_spectrum(k)
    A = matgen.random_sym_csr(10000, 0.01, 20261015, plant)
    B = matgen.random_sym_csr(10000, 0.01, 20261015, plant)
    assert (A - A.T).nnz == 0 and (A != B).nnz == 0
    assert abs(A.nnz / 10000 - 2 * 0.01 * 10000) < 5   # ~200 per row (R + R^T)
    omega = np.random.default_rng(1).standard_normal((10000, 8))
    r = o.RBL_gpu_semantics(A, k, 8, omega=omega, qr_mode="posdiag")
    assert r.converged
    assert np.abs(r.D - plant[:k]).max() < 1.0
    res = np.linalg.norm(A @ r.V - r.V * r.D, axis=0) / np.abs(r.D)
    assert res.max() < 1e-8
