"""GPU: the CSR SpMM kernels (global gather and LDS window) against SciPy's A @ X.

Floating-point tolerance: every output element within 1e-13 * (|A| |X|) of the fp64 SciPy
product (the kernels only reorder the fp64 sums)."""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import matgen

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rbl():
    import rbl as _r
    return _r


def _check(A, Y, X):
    ref = A @ X
    bound = (abs(A) @ np.abs(X)) * 1e-13 + 1e-300
    assert np.all(np.abs(Y - ref) <= bound), np.max(np.abs(Y - ref) / bound)


def _rand_sym(n, density, seed, empty_rows=()):
    R = sp.random(n, n, density=density, random_state=seed, format="csr")
    A = (R + R.T).tolil()
    for r in empty_rows:
        A[r, :] = 0
        A[:, r] = 0
    return sp.csr_matrix(A)


@pytest.mark.parametrize("b", [1, 5, 8, 16, 32, 64])
@pytest.mark.parametrize("variant", [0, 1, 2, 3, 5])
def test_spmm_hashwindow(rbl, b, variant):
    """RBL_OPT_SPMM_KERNEL takes the kernel ids rbl_spmm_kernel_for reports: 1 = gather,
    2 = LDS window (DPP), 3 = LDS-densified band on MFMA, 5 = band tiles (MFMA operand order,
    spmm_bt.hip), 0 = auto."""
    A = matgen.hashwindow_csr(7000, 64, 0.7734, 5, matgen.planted_spectrum(10))
    X = np.random.default_rng(b).standard_normal((A.shape[0], b))
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        ctx.set_option(2, variant)
        k = ctx.spmm_kernel_for(b)
        if b in (16, 32):
            assert k == {0: 5, 1: 1, 2: 2, 3: 3, 5: 5}[variant]   # the kernel under test runs
        else:
            assert k == 1
        Y = ctx.apply(X)
    _check(A, Y, X)


@pytest.mark.parametrize("b", [16, 32])
def test_spmm_window_ragged_and_partial_tiles(rbl, b):
    """n not a multiple of the 16-row tile, narrow and wide windows, rows of very different
    lengths and a band that grows then shrinks."""
    for n, W, p in [(1001, 3, 0.9), (333, 100, 0.3), (4099, 64, 1.0), (17, 8, 0.5)]:
        A = matgen.hashwindow_csr(n, W, p, n)
        X = np.random.default_rng(n).standard_normal((n, b))
        with rbl.Context(0) as ctx:
            ctx.set_matrix(A)
            Y = ctx.apply(X)
            k = ctx.spmm_kernel_for(b)
        _check(A, Y, X)
        tile_nnz = np.diff(A.indptr[np.r_[np.arange(0, n, 16), n]]).max()
        if W <= 64 and tile_nnz <= 2048:     # the window kernel's metadata cap per tile
            assert k in (2, 3, 5, 7), (n, W)   # (7: the column panels, ahead of the window)
        if tile_nnz > 2048:
            assert k in (1, 3, 5, 6), (n, W)


@pytest.mark.parametrize("b", [16, 32])
@pytest.mark.parametrize("variant", [2, 3, 5])
def test_spmm_window_kernels_ragged(rbl, b, variant):
    """Both LDS kernels forced, on ragged tiles / narrow and wide bands / dense bands."""
    for n, W, p in [(1001, 3, 0.9), (333, 60, 0.5), (4099, 64, 1.0), (17, 8, 0.5), (2000, 30, 0.2)]:
        A = matgen.hashwindow_csr(n, W, p, n + 7)
        X = np.random.default_rng(n).standard_normal((n, b))
        with rbl.Context(0) as ctx:
            ctx.set_matrix(A)
            ctx.set_option(2, variant)
            Y = ctx.apply(X)
        _check(A, Y, X)


@pytest.mark.parametrize("b", [8, 16, 32])
def test_spmm_general_pattern_and_empty_rows(rbl, b):
    """Random (R-MAT-like, unbanded) pattern: the gather kernel; empty rows give zero rows."""
    A = _rand_sym(3000, 0.01, 3, empty_rows=(0, 5, 2999))
    X = np.random.default_rng(1).standard_normal((3000, b))
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        # segmented / plain gather; at b = 32 this small pattern also passes the column panels'
        # reuse rule (every staged Q row read >= 4 times), so either may be chosen
        assert ctx.spmm_kernel_for(b) in ({6, 7} if b == 32 else {6} if b == 16 else {1})
        Y = ctx.apply(X)
    _check(A, Y, X)
    assert np.all(Y[[0, 5, 2999]] == 0)


def test_spmm_window_and_gather_agree_in_lanczos(rbl):
    """The whole block step is insensitive to the SpMM kernel choice (1e-12 on A_i)."""
    A = matgen.hashwindow_csr(6000, 64, 0.7734, 9, matgen.planted_spectrum(10))
    out = []
    for variant in (1, 2, 3, 5):
        with rbl.Context(0) as ctx:
            ctx.set_matrix(A)
            ctx.set_option(2, variant)
            _, _, info = rbl.lanczos(ctx, 10, 32, seed=4, check=False, max_steps=6, trace=True,
                                     ritz=False)
            out.append(info)
    for a1, a2 in zip(out[0].trace_A, out[1].trace_A):
        assert np.abs(a1 - a2).max() <= 1e-12 * np.abs(a1).max()


@pytest.mark.parametrize("b", [16, 32])
@pytest.mark.parametrize("n,W,p,ng", [(7000, 64, 0.7734, 9), (5003, 30, 0.9, 5), (300, 60, 1.0, 9),
                                      (100, 30, 1.0, 5), (17, 8, 0.5, 0), (4099, 64, 0.2, 0)])
def test_spmm_band_tiles(rbl, n, W, p, ng, b):
    """Band-tile kernel (spmm_bt.hip) at both band widths (H = 32: NG = 5 groups, H = 64: 9),
    ragged last tiles and matrices smaller than one round; a sparse band (p = 0.2) must NOT
    take it (its dense tiles would stream 3x the CSR bytes)."""
    A = matgen.hashwindow_csr(n, W, p, n + 3)
    X = np.random.default_rng(n).standard_normal((n, b))
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        k = ctx.spmm_kernel_for(b)
        Y = ctx.apply(X)
    assert (k == 5) == (ng > 0), (k, ng)
    _check(A, Y, X)


@pytest.mark.parametrize("b", [16, 32])
@pytest.mark.parametrize("variant", [0, 6])
def test_spmm_segmented_long_rows(rbl, b, variant):
    """Segmented gather (kernel id 6): an arrow matrix whose 3 hub rows/columns
    touch every row (20,000 nonzeros each: 5 segments of 4,096 each, summed in order by the
    fixup kernel) beside short random rows, empty rows and the fused 3-term epilogue path
    through a short Lanczos trace."""
    n = 20000
    R = sp.random(n, n, density=2e-4, random_state=5, format="csr")
    hub = sp.lil_matrix((n, n))
    hub[[0, 7, 19999], :] = np.random.default_rng(1).standard_normal((3, n))
    A = R + R.T + hub + hub.T
    A = A.tolil()
    A[123, :] = 0
    A[:, 123] = 0
    A = sp.csr_matrix(A)
    X = np.random.default_rng(b).standard_normal((n, b))
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        ctx.set_option(2, variant)
        assert ctx.spmm_kernel_for(b) == 6
        Y = ctx.apply(X)
    _check(A, Y, X)
    assert np.all(Y[123] == 0)


def test_spmm_segmented_and_gather_agree_in_lanczos(rbl):
    """Epilogue + long-row fixup inside a block step: kernels 6 and 1 give the same A_i."""
    from oracle import matgen as mg
    A = mg.rmat_csr(16000, 14, 1_200_000, 3, mg.planted_spectrum(5))
    assert np.diff(A.indptr).max() > 4096     # long rows present
    out = []
    for variant in (1, 6):
        with rbl.Context(0) as ctx:
            ctx.set_matrix(A)
            ctx.set_option(2, variant)
            _, _, info = rbl.lanczos(ctx, 5, 32, seed=4, check=False, max_steps=6, trace=True,
                                     ritz=False)
            out.append(info)
    for a1, a2 in zip(out[0].trace_A, out[1].trace_A):
        assert np.abs(a1 - a2).max() <= 1e-12 * np.abs(a1).max()



# ---- column-panel CSR kernel (spmm_panel.hip, kernel id 7, b = 32) ----------------------------
PANEL_CASES = [(50003, 300, 0.165), (20000, 1024, 0.0483), (3000, 2048, 0.024), (70001, 130, 1.0),
               (257, 100, 0.5), (40000, 90, 0.55)]


@pytest.mark.parametrize("n,W,p", PANEL_CASES)
def test_spmm_column_panels(rbl, n, W, p):
    """Wide bands (half-width 90 .. 2048, beyond the band tiles' 64): the automatic choice is
    the column-panel kernel, and U = A X within 1e-13 |A||X| of SciPy — ragged last blocks
    (n not a multiple of 256), a window wider than the matrix, rows with up to 261 nonzeros in
    one 256-row panel (the chunk reload path), a matrix of one block and one row."""
    A = matgen.hashwindow_csr(n, W, p, n + 3, matgen.planted_spectrum(5))
    X = np.random.default_rng(n).standard_normal((n, 32))
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        assert ctx.spmm_kernel_for(32) == 7, (n, W)
        Y = ctx.apply(X)
    _check(A, Y, X)


@pytest.mark.parametrize("case", ["random", "empty_rows", "planted_diag"])
def test_spmm_column_panels_forced(rbl, case):
    """Kernel 7 forced (RBL_OPT_SPMM_KERNEL) on patterns it would not be chosen for: a random
    unbanded matrix (every block spans every panel), empty rows and columns (zero rows of U),
    a diagonal matrix (one panel per block, one entry per row)."""
    n = 5000
    if case == "random":
        A = _rand_sym(n, 0.002, 9)
    elif case == "empty_rows":
        A = _rand_sym(n, 0.004, 4, empty_rows=(0, 255, 256, 4999))
    else:
        A = sp.diags(np.arange(1.0, n + 1.0)).tocsr()
    X = np.random.default_rng(3).standard_normal((n, 32))
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        ctx.set_option(2, 7)
        assert ctx.spmm_kernel_for(32) == 7
        Y = ctx.apply(X)
    _check(A, Y, X)
    if case == "empty_rows":
        assert np.all(Y[[0, 255, 256, 4999]] == 0)


def test_spmm_column_panels_in_lanczos(rbl):
    """Inside block steps (the 3-term epilogue U -= Q_{i-1} B_i^T fused in the kernel,
    RBL_gpu.jl:176-177): 8 steps on a half-width-700 band against the oracle's A_i / B_{i+1}
    (1e-9 relative, as the other trace tests) and against the plain gather kernel (1e-12)."""
    from oracle import rbl_oracle as o
    n, W, b = 30011, 700, 32
    A = matgen.hashwindow_csr(n, W, 0.07, 13, matgen.planted_spectrum(10))
    omega = np.random.default_rng(5).standard_normal((n, b))
    steps = 8
    ref = o.RBL_gpu_semantics(A, 10, b, omega=omega, qr_mode="posdiag", reorth_mode="cgs",
                              check=False, max_steps=steps, trace=True)
    out = {}
    for kernel in (0, 1):
        with rbl.Context(0) as ctx:
            ctx.set_matrix(A)
            ctx.set_option(2, kernel)
            assert ctx.spmm_kernel_for(b) == (7 if kernel == 0 else 1)
            _, _, info = rbl.lanczos(ctx, 10, b, omega=omega, check=False, max_steps=steps,
                                     trace=True, ritz=False)
        out[kernel] = info
    for i in range(steps):
        Ar, Br = ref.trace["A"][i], ref.trace["B"][i]
        Ag, Bg = out[0].trace_A[i], out[0].trace_B[i]
        assert np.abs(Ag - Ar).max() <= 1e-9 * np.abs(Ar).max(), i
        assert np.abs(Bg - Br).max() <= 1e-9 * np.abs(Br).max(), i
        for x, y in ((Ag, out[1].trace_A[i]), (Bg, out[1].trace_B[i])):
            assert np.abs(x - y).max() <= 1e-12 * np.abs(y).max(), i
