"""CPU: the oracle and the host-side generators against the committed golden fixtures
(tests/golden/, made by tests/golden/make_golden.py).

Tolerances: eigenvalues 1e-12 relative (same algorithm, BLAS threading may reorder sums),
per-step A_i / B_i 1e-10 relative, Ritz vectors 1 - |v.v'| < 1e-10; the reference's own
algorithm choices (Householder QR, ascending-j block MGS) agree with the HIP path's choices
(positive-diagonal QR, block CGS) to 1e-10 on the eigenvalues; known-answer suites 1e-13
(test.jl:16-50); generators bit-exact.
"""
import os

import numpy as np
import scipy.sparse as sp

from oracle import matgen
from oracle import rbl_oracle as o

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(G, name))  # allow_pickle=False (default)


def c1():
    z = load("golden_c1.npz")
    n = int(z["n"])
    A = sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=(n, n))
    return z, A


def test_c1_fixture_is_the_documented_input():
    import importlib.util
    spec = importlib.util.spec_from_file_location("make_golden", os.path.join(G, "make_golden.py"))
    mg = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mg)
    z, A = c1()
    A2 = mg.c1_matrix()
    assert (A != A2).nnz == 0
    assert abs(A - A.T).max() == 0.0


def test_oracle_reproduces_c1():
    z, A = c1()
    k, b = int(z["k"]), int(z["b"])
    r = o.RBL_gpu_semantics(A, k, b, omega=z["omega"], qr_mode="posdiag", reorth_mode="cgs")
    assert r.converged and r.iters == int(z["iters"])
    assert np.max(np.abs(r.D - z["D"]) / np.abs(z["D"])) < 1e-12
    dots = np.abs(np.sum(r.V * z["V"], axis=0))
    assert np.all(1 - dots < 1e-10)
    t = o.RBL_gpu_semantics(A, k, b, omega=z["omega"], qr_mode="posdiag", reorth_mode="cgs",
                            check=False, max_steps=8, trace=True).trace
    for a, ag in zip(t["A"], z["trace_A"]):
        assert np.abs(a - ag).max() <= 1e-10 * np.abs(ag).max()
    for bb, bg in zip(t["B"], z["trace_B"]):
        assert np.abs(bb - bg).max() <= 1e-10 * np.abs(bg).max()


def test_reference_choices_agree_on_c1():
    """Householder + ascending-j MGS (the reference) vs posdiag CholQR + block CGS (HIP)."""
    z, _ = c1()
    assert np.max(np.abs(z["D_reference_choices"] - z["D"]) / np.abs(z["D"])) < 1e-10


def test_c1_eigenpairs_are_eigenpairs():
    z, A = c1()
    V, D = z["V"], z["D"]
    res = np.linalg.norm(A @ V - V * D[None, :], axis=0) / np.abs(D)
    assert np.all(res < 1e-7)
    assert np.all(np.diff(np.abs(D)) <= 0)          # descending |lambda| (P11)


def test_hashwindow_generators_bit_exact():
    from rbl import _lib
    z = load("golden_hashwindow.npz")
    n, W, p, seed, plant = int(z["n"]), int(z["W"]), float(z["p"]), int(z["seed"]), z["plant"]
    for tag in ("head", "tail"):
        r0, r1 = (int(x) for x in z[f"{tag}_rows"])
        M = matgen.hashwindow_csr(n, W, p, seed, plant, r0, r1)
        assert np.array_equal(M.indptr, z[f"{tag}_indptr"])
        assert np.array_equal(M.indices, z[f"{tag}_indices"])
        assert np.array_equal(M.data.view(np.uint64), z[f"{tag}_data"].view(np.uint64))
        rp, col, val = _lib.hashwindow_rows_host(n, W, p, seed, plant, r0, r1)
        assert np.array_equal(rp, z[f"{tag}_indptr"])
        assert np.array_equal(col, z[f"{tag}_indices"])
        assert np.array_equal(val.view(np.uint64), z[f"{tag}_data"].view(np.uint64))


def test_known_answer_fixture():
    z = load("golden_known_answer.npz")
    for name, (gen, ns, k, b) in o.KNOWN_ANSWER_SUITES.items():
        for n in ns:
            _, eig = gen(n, k)
            assert np.array_equal(eig, z[f"{name}_{n}_expected"])
            err = np.abs(z[f"{name}_{n}_oracle"] - eig) / eig
            assert np.linalg.norm(err) < o.KNOWN_ANSWER_TOL
