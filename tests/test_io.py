"""CPU: the Matrix Market / .mat loaders (benchmark.jl:21-28 inputs) round-trip symmetric
matrices exactly and reject non-symmetric ones."""
import os

import numpy as np
import pytest
import scipy.io
import scipy.sparse as sp

from oracle import matgen


@pytest.fixture(scope="module")
def io():
    from rbl import io as _io
    return _io


def test_matrix_market_symmetric_roundtrip(io, tmp_path):
    A = matgen.hashwindow_csr(300, 5, 0.6, 3)
    p = os.path.join(tmp_path, "a.mtx")
    scipy.io.mmwrite(p, sp.coo_matrix(A), symmetry="symmetric", precision=17)
    B = io.load_matrix(p)
    assert B.format == "csc" and B.dtype == np.float64
    assert abs(B - A).max() == 0.0


def test_mat_problem_struct(io, tmp_path):
    A = matgen.hashwindow_csr(200, 4, 0.5, 9)
    p = os.path.join(tmp_path, "ldoor_like.mat")
    scipy.io.savemat(p, {"Problem": {"A": sp.csc_matrix(A), "name": "test"}})
    B = io.load_matrix(p)
    assert abs(B - A).max() == 0.0


def test_rejects_nonsymmetric(io, tmp_path):
    A = sp.random(50, 50, density=0.1, random_state=1, format="coo")
    p = os.path.join(tmp_path, "g.mtx")
    scipy.io.mmwrite(p, A)
    with pytest.raises(ValueError):
        io.load_matrix(p)
