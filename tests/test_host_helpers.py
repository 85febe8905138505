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
