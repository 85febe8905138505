"""GPU: the memory plan around the hot path — what the reference's
`gpu_buffer_size` / `matrix_size` / `blocksize` (RBL_gpu.jl:8-27, 95-104) decide, made explicit:

  * RBL_OPT_KEEP_CSR = 0 releases the device CSR once the band tiles are built (12 B per
    nonzero of HBM returned to the Krylov basis: what lets n = 5e7 run on one GPU).  The run
    must be bit-identical to the one that keeps the CSR; paths that need the CSR fail loudly;
  * rbl_ritz splits the Ritz columns into chunks of <= 64 (RBL_gpu.jl:110-125): k > 64 must
    equal [Q_1..Q_m] S formed on the host (fp64, 1e-13 relative to |Q||S|);
  * rbl_comm_info reports the transport's own rank count.
"""
import numpy as np
import pytest

from oracle import matgen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rbl():
    import rbl as _r
    return _r


def band_matrix(n=6000, k=10, seed=5):
    return matgen.hashwindow_csr(n, 64, 0.7734, seed, matgen.planted_spectrum(k))


@pytest.mark.parametrize("b,bits", [(32, 64), (16, 64), (32, 32)])
def test_keep_csr_off_bit_identical(rbl, b, bits):
    A = band_matrix()
    omega = np.random.default_rng(b).standard_normal((A.shape[0], b))
    out = []
    for keep in (1, 0):
        with rbl.Context(0) as ctx:
            ctx.set_option(rbl._lib.RBL_OPT_KEEP_CSR, keep)
            ctx.set_matrix(A)
            assert ctx.spmm_kernel_for(b) == 5
            D, V, info = rbl.lanczos(ctx, 10, b, omega=omega, trace=True, basis_bits=bits)
            out.append((D, V, info))
            if not keep:
                with pytest.raises(rbl.RBLError):
                    ctx.get_matrix_csr()
                with pytest.raises(rbl.RBLError):   # only the band tiles remain: b = 8 cannot run
                    ctx.apply(np.ones((A.shape[0], 8)))
    (D1, V1, i1), (D0, V0, i0) = out
    assert i1.converged and i0.converged and i1.iters == i0.iters
    assert np.array_equal(D1, D0) and np.array_equal(V1, V0)
    for a1, a0 in zip(i1.trace_A + i1.trace_B, i0.trace_A + i0.trace_B):
        assert np.array_equal(a1, a0)


def test_keep_csr_off_without_band_tiles_keeps_csr(rbl):
    """A pattern the band tiles cannot hold (unbanded): the option has nothing to release to."""
    A = matgen.rmat_csr(4096, 12, 40000, 3, matgen.planted_spectrum(4))
    with rbl.Context(0) as ctx:
        ctx.set_option(rbl._lib.RBL_OPT_KEEP_CSR, 0)
        ctx.set_matrix(A)
        assert ctx.spmm_kernel_for(16) != 5
        rp, ci, v = ctx.get_matrix_csr()
        assert np.array_equal(rp, A.indptr) and np.array_equal(v, A.data)
        X = np.random.default_rng(0).standard_normal((A.shape[0], 8))
        assert np.abs(ctx.apply(X) - A @ X).max() <= 1e-12 * abs(A).sum(axis=1).max() * np.abs(X).max()


@pytest.mark.parametrize("b,k,bits", [(32, 150, 64), (16, 70, 64), (32, 100, 32)])
def test_ritz_chunked_columns(rbl, b, k, bits):
    A = band_matrix(3000)
    omega = np.random.default_rng(1).standard_normal((A.shape[0], b))
    steps = 6
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        rbl.lanczos(ctx, 10, b, omega=omega, check=False, max_steps=steps, ritz=False,
                    basis_bits=bits)
        Q = np.hstack([ctx.get_block(j) for j in range(1, steps + 1)])
        S = np.asfortranarray(np.random.default_rng(4).standard_normal((steps * b, k)))
        V = ctx.ritz(steps, k, S)
    ref = Q @ S
    assert V.shape == ref.shape
    assert np.abs(V - ref).max() <= 1e-13 * np.abs(Q).max() * np.abs(S).sum(axis=0).max()


def test_comm_info(rbl):
    with rbl.Context(0) as ctx:
        assert ctx.comm_info() == {"nranks": 1, "rank": 0, "transport": "none"}
    from test_gpu_multirank import run_ranks

    def fn(ctx, r):
        return ctx.comm_info()

    infos = run_ranks(rbl, 3, fn)
    assert [d["rank"] for d in infos] == [0, 1, 2]
    assert all(d["nranks"] == 3 and d["transport"] == "local" for d in infos)
