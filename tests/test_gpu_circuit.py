"""GPU: the circuit-like generator (BASELINE config 3's shape: G3_circuit, n = 1,585,478,
7.66 M nonzeros; the real file is not in the image) on the device.

rbl_gen_matrix_circuit must build the NumPy restatement's matrix (oracle/matgen.py
circuit_like_csr: 5-point weighted Laplacian, hash-kept edges, Feistel node scatter) bit for bit
— integer structure and fp64 values — on one rank and on the row slices of several in-process
ranks; the SpMM on it (segmented gather, no band) is checked against SciPy."""
import numpy as np
import pytest

from oracle import matgen
from test_gpu_multirank import run_ranks

pytestmark = pytest.mark.gpu

CASE = dict(n=20011, width=137, seed=5)


@pytest.fixture(scope="module")
def rbl():
    import rbl as _r
    return _r


def _csr_equal(ref, rowptr, col, val):
    assert np.array_equal(ref.indptr, rowptr)
    assert np.array_equal(ref.indices, col)
    assert np.array_equal(ref.data, val)


@pytest.mark.parametrize("n,width", [(20011, 137), (1, 1), (7, 3), (4096, 64)])
def test_circuit_generator_bit_exact(rbl, n, width):
    plant = matgen.planted_spectrum(3)
    ref = matgen.circuit_like_csr(n, 5, plant, width=width)
    with rbl.Context(0) as ctx:
        ctx.gen_circuit(n, 5, plant, width=width)
        assert ctx.matrix_info() == (n, 0, n, ref.nnz)
        _csr_equal(ref, *ctx.get_matrix_csr())


def test_circuit_generator_g3_shape(rbl):
    """The defaults give G3_circuit's n and ~its nonzero count, without a band."""
    with rbl.Context(0) as ctx:
        ctx.gen_circuit(plant=matgen.planted_spectrum(20))
        n, r0, r1, nnz = ctx.matrix_info()
        assert n == matgen.G3_CIRCUIT_N and abs(nnz - matgen.G3_CIRCUIT_NNZ) < 0.001 * nnz
        assert ctx.spmm_kernel_for(16) == 6
        ref = matgen.circuit_like_csr(plant=matgen.planted_spectrum(20))
        _csr_equal(ref, *ctx.get_matrix_csr())


@pytest.mark.parametrize("P", [2, 3])
def test_circuit_generator_ranks(rbl, P):
    plant = matgen.planted_spectrum(3)
    full = matgen.circuit_like_csr(CASE["n"], CASE["seed"], plant, width=CASE["width"])

    def fn(ctx, r):
        ctx.gen_circuit(CASE["n"], CASE["seed"], plant, width=CASE["width"])
        _, r0, r1, _ = ctx.matrix_info()
        return r0, r1, ctx.get_matrix_csr()

    parts = run_ranks(rbl, P, fn)
    assert parts[0][0] == 0 and parts[-1][1] == CASE["n"]
    for r0, r1, csr in parts:
        _csr_equal(full[r0:r1], *csr)


@pytest.mark.parametrize("b", [16, 32])
def test_circuit_spmm(rbl, b):
    A = matgen.circuit_like_csr(CASE["n"], CASE["seed"], width=CASE["width"])
    X = np.random.default_rng(b).standard_normal((A.shape[0], b))
    with rbl.Context(0) as ctx:
        ctx.gen_circuit(CASE["n"], CASE["seed"], width=CASE["width"])
        Y = ctx.apply(X)
    ref = A @ X
    bound = (abs(A) @ np.abs(X)) * 1e-13 + 1e-300
    assert np.all(np.abs(Y - ref) <= bound)
