"""CPU: the product's host helpers (rbl.host, common.jl restated) against the oracle's."""
import numpy as np

from oracle import rbl_oracle as o


def test_tband_matches_oracle_insert():
    from rbl.host import TBand
    rng = np.random.default_rng(2)
    b, m = 5, 6
    tb = TBand(b, m)
    T = None
    for i in range(m):
        A = rng.standard_normal((b, b))
        A = A + A.T
        B = np.triu(rng.standard_normal((b, b)))
        tb.insert_A(A)
        T = o.insertA(A, b) if T is None else np.hstack([T, o.insertA(A, b)])
        if i < m - 1:
            tb.insert_B(B, i + 1)
            o.insertB(B, T, b, i + 1)
    assert np.array_equal(tb.view(), T)


def test_dsbev_sort_convergence_match_oracle():
    from rbl import host
    rng = np.random.default_rng(3)
    b, N = 4, 40
    T = rng.standard_normal((b + 1, N))
    d1, v1 = host.dsbev(T)
    d2, v2 = o.dsbev(T)
    assert np.array_equal(d1, d2) and np.array_equal(v1, v2)
    s1 = host.sort_eig_abs(d1, v1, 7)
    s2 = o.sort_eig_abs(d2, v2, 7)
    assert np.array_equal(s1[0], s2[0]) and np.array_equal(s1[1], s2[1])
    B = np.triu(rng.standard_normal((b, b))) * 1e-9
    assert host.check_convergence(B, s1[1], b, 7, 1e-7) == o.check_convergence(B, s2[1], b, 7, 1e-7)


def test_large_band_eigensolve_matches_reference_routine():
    """From N = 256 on the host uses dsbevd: the same eigenvalues as the reference's dsbev to
    rounding, eigenvectors orthonormal with small residuals, and the same top-k selection."""
    from rbl import host
    rng = np.random.default_rng(4)
    b, N = 32, 512
    T = rng.standard_normal((b + 1, N))
    d1, v1 = host.dsbev(T)
    d2, v2 = o.dsbev(T)
    scale = np.abs(d2).max()
    assert np.abs(d1 - d2).max() < 1e-12 * scale
    full = np.zeros((N, N))
    for r in range(b + 1):  # lower band storage -> dense symmetric
        idx = np.arange(N - r)
        full[idx + r, idx] = T[r, : N - r]
        full[idx, idx + r] = T[r, : N - r]
    assert np.abs(full @ v1 - v1 * d1).max() < 1e-11 * scale
    assert np.abs(v1.T @ v1 - np.eye(N)).max() < 1e-11
    s1 = host.sort_eig_abs(d1, v1, 20)
    s2 = o.sort_eig_abs(d2, v2, 20)
    assert np.abs(s1[0] - s2[0]).max() < 1e-12 * scale


def test_topk_eigensolve_matches_reference_selection():
    """The loop's k largest-|lambda| pairs (rbl.host.eig_topk: dsyevr on the 2k end pairs from
    N = 512 on) equal the reference's dsbev + sort_eig_abs (common.jl:36-54): eigenvalues to
    rounding, vectors up to sign, the same convergence decision; both spectrum ends compete."""
    from rbl import host
    rng = np.random.default_rng(6)
    for N, b, k, shift in [(512, 32, 20, 0.0), (640, 16, 20, -40.0), (768, 32, 7, 40.0)]:
        T = rng.standard_normal((b + 1, N))
        T[0] += shift * np.sin(np.arange(N))      # large eigenvalues of both signs
        d1, v1 = host.eig_topk(T, k)
        d2, v2 = o.sort_eig_abs(*o.dsbev(T), k)
        scale = np.abs(d2).max()
        assert np.abs(d1 - d2).max() < 1e-12 * scale
        assert (1 - np.abs((v1 * v2).sum(axis=0))).max() < 1e-10
        B = np.triu(rng.standard_normal((b, b)))
        for tol in (1e-3, 1e2):
            assert host.check_convergence(B, v1, b, k, tol) == o.check_convergence(B, v2, b, k, tol)


def test_fix_signs_makes_ritz_coefficients_solver_independent():
    """The top-k path and dsbev may return eigenvectors of opposite signs; after fix_signs the
    coefficient columns (hence V = [Q] S) agree entry for entry."""
    from rbl.host import eig_topk, fix_signs, sort_eig_abs
    from scipy.linalg import lapack
    rng = np.random.default_rng(11)
    b, N, k = 8, 640, 10
    T = rng.standard_normal((b + 1, N))
    T[0] += np.linspace(-50, 60, N)
    w, z, info = lapack.dsbev(T, compute_v=1, lower=1)
    D1, S1 = sort_eig_abs(w, z, k)
    D2, S2 = eig_topk(T, k)
    assert np.allclose(D1, D2, rtol=1e-12, atol=0)
    F1, F2 = fix_signs(S1), fix_signs(S2)
    assert np.abs(F1 - F2).max() < 1e-9
    assert np.all(F1[np.argmax(np.abs(F1), axis=0), np.arange(k)] > 0)
    neg = fix_signs(-S1)
    assert np.array_equal(neg, F1)


def test_speculation_rule_from_residual_history():
    """rbl.lanczos's speculate="auto": run ahead of a check by 4 steps when the geometric
    extrapolation of the earlier checks' max residual bounds stays >= 100x above the tolerance,
    by 2 between 5x and 100x, by 1 between 1x and 5x, else not; the residual bounds are common.jl:56-65's norms
    (check_convergence is their all-below-tol test)."""
    from rbl.host import check_convergence, residual_norms, speculation_depth
    tol = 1e-7
    assert speculation_depth([], tol) == 0 and speculation_depth([1.0], tol) == 0
    assert speculation_depth([1e-1, 1e-2], tol) == 4           # next ~1e-3
    assert speculation_depth([1e-3, 2e-3], tol) == 4           # growth clamped: next ~2e-3
    assert speculation_depth([2.8e-3, 4.0e-5], tol) == 2       # next ~5.7e-7 (C4a slow, check 24)
    assert speculation_depth([1e-4, 4e-6], tol) == 1           # next ~1.6e-7: within 5x of tol
    assert speculation_depth([4.0e-5, 6.0e-7], tol) == 0       # next ~9e-9: expected to converge
    assert speculation_depth([0.0, 1e-3], tol) == 0 and speculation_depth([1.0, float("nan")], tol) == 0
    # the C4a slow-spectrum bounds of profiles/r05_ttk_probe_b26.log: 4, 4, 4, 2, 0 from check 3 on
    r = [4.8e+00, 2.5e+00, 1.9e-01, 2.8e-03, 4.0e-05, 6.0e-07, 8.9e-09]
    assert [speculation_depth(r[:j], tol) for j in range(2, 7)] == [4, 4, 4, 2, 0]
    rng = np.random.default_rng(0)
    b, k = 4, 3
    B, S = rng.standard_normal((b, b)), rng.standard_normal((20, 6))
    r = residual_norms(B, S, b, k)
    assert r.shape == (k,) and np.allclose(r, np.linalg.norm(B @ S[-b:, :k], axis=0))
    assert check_convergence(B, S, b, k, r.max() * 1.001) and not check_convergence(B, S, b, k, r.max() * 0.999)


def test_eigensolve_allocates_without_hugepage_advice():
    """eig_topk's arrays are allocated under small_pages(): NumPy's MADV_HUGEPAGE advice is off
    inside (THP compaction on their first touch stalled the GPU) and restored after,
    also when the solve raises; the dense top-k path still matches dsbev's eigenvalues."""
    import pytest
    from rbl import host
    if host._np_madvise_hugepage is None:
        pytest.skip("this NumPy has no madvise switch")
    from numpy._core.multiarray import _get_madvise_hugepage
    before = _get_madvise_hugepage()
    seen = []
    real = host._eig_topk_dense

    def spy(T, k):
        seen.append(_get_madvise_hugepage())
        return real(T, k)

    rng = np.random.default_rng(3)
    b, m, k = 16, 40, 5
    T = host.TBand(b, m)
    for j in range(1, m + 1):
        a = rng.standard_normal((b, b))
        T.insert_A(a + a.T)
        T.insert_B(np.triu(rng.standard_normal((b, b))), j)
    host._eig_topk_dense = spy
    try:
        D, _ = host.eig_topk(T.view(), k)
    finally:
        host._eig_topk_dense = real
    assert seen == [False] and _get_madvise_hugepage() == before
    Dr, _ = host.sort_eig_abs(*host.dsbev(T.view()), k)
    assert np.allclose(np.sort(D), np.sort(Dr), rtol=1e-12)
    try:
        with host.small_pages():
            raise RuntimeError("x")
    except RuntimeError:
        pass
    assert _get_madvise_hugepage() == before
