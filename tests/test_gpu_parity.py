"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on the same inputs.

Tolerances (north star / SURVEY §8(c)):
  * eigenvalues  |lambda_gpu - lambda_oracle| / |lambda| < 1e-10;
  * reference known-answer suites (test.jl): relative error norm < 1e-13;
  * eigenvectors 1 - |v_gpu^T v_oracle| < 1e-8 and ||A v - lambda v|| / |lambda| < 1e-7;
  * per-step A_i, B_{i+1} (CholQR R has a non-negative diagonal, so the oracle runs with
    qr_mode="posdiag"): relative 1e-9 over the first steps.
"""
import numpy as np
import pytest

from oracle import matgen
from oracle import rbl_oracle as o

pytestmark = pytest.mark.gpu

EIG_TOL = 1e-10
VEC_TOL = 1e-8
RES_TOL = 1e-7


@pytest.fixture(scope="module")
def rbl():
    import rbl as _r
    return _r


def c1_matrix(n=10000, k=10, W=64, seed=20261015):
    """symmetric hash-window + planted top spectrum."""
    p = min(1.0, 0.01 * n / (2 * W)) if n <= 2 * W * 100 else 0.7734
    return matgen.hashwindow_csr(n, W, p, seed, matgen.planted_spectrum(k))


def test_device_generator_bit_exact(rbl):
    n, W, p, seed = 20000, 64, 0.7734, 99
    plant = matgen.planted_spectrum(10)
    with rbl.Context(0) as ctx:
        ctx.gen_hashwindow(n, W, p, seed, plant)
        rp, col, val = ctx.get_matrix_csr()
    A = matgen.hashwindow_csr(n, W, p, seed, plant)
    assert np.array_equal(rp, A.indptr)
    assert np.array_equal(col.astype(np.int64), A.indices)
    assert np.array_equal(val, A.data)


@pytest.mark.parametrize("b", [1, 5, 8, 16, 32])
def test_first_steps_trace(rbl, b):
    A = c1_matrix(4000, 10)
    n = A.shape[0]
    omega = np.random.default_rng(b).standard_normal((n, b))
    steps = 6
    ref = o.RBL_gpu_semantics(A, 10, b, omega=omega, qr_mode="posdiag", reorth_mode="cgs",
                              check=False, max_steps=steps, trace=True)
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        _, _, info = rbl.lanczos(ctx, 10, b, omega=omega, check=False, max_steps=steps,
                                 trace=True, ritz=False)
    assert len(info.trace_A) == len(ref.trace["A"]) == steps
    for i in range(steps):
        Ar, Br = ref.trace["A"][i], ref.trace["B"][i]
        Ag, Bg = info.trace_A[i], info.trace_B[i]
        sa = np.abs(Ar).max()
        sb = np.abs(Br).max()
        assert np.abs(Ag - Ar).max() <= 1e-9 * sa, (i, np.abs(Ag - Ar).max(), sa)
        assert np.abs(Bg - Br).max() <= 1e-9 * sb, (i, np.abs(Bg - Br).max(), sb)


@pytest.mark.parametrize("b", [16, 32])
def test_long_trace_every_panel_remainder(rbl, b):
    """16 block steps (partial reorth over nW = 2 .. 14 basis panels: every remainder of the
    4-panel groups of k_gram44, including the tail groups that cover 2 or 4 splits' rows)
    against the oracle's per-step A_i, B_{i+1}; a slowly decaying spectrum keeps the blocks
    away from rounding-dominated directions.  Relative 1e-8 of the block's max entry."""
    n = 3000
    rng = np.random.default_rng(11)
    import scipy.sparse as sp
    R = sp.random(n, n, density=0.004, random_state=5, format="csr")
    A = (R + R.T + sp.diags(np.linspace(1.0, 3.0, n))).tocsr()
    omega = rng.standard_normal((n, b))
    steps = 16
    ref = o.RBL_gpu_semantics(A, 10, b, omega=omega, qr_mode="posdiag", reorth_mode="cgs",
                              check=False, max_steps=steps, trace=True)
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        _, _, info = rbl.lanczos(ctx, 10, b, omega=omega, check=False, max_steps=steps,
                                 trace=True, ritz=False)
    assert len(info.trace_A) == steps
    for i in range(steps):
        Ar, Br = ref.trace["A"][i], ref.trace["B"][i]
        da = np.abs(info.trace_A[i] - Ar).max() / np.abs(Ar).max()
        db = np.abs(info.trace_B[i] - Br).max() / np.abs(Br).max()
        assert da < 1e-8 and db < 1e-8, (i, da, db)


@pytest.mark.parametrize("order,b", [(0, 8), (1, 8), (0, 16), (1, 16), (0, 32)])
def test_eigenpairs_c1(rbl, order, b):
    """C1 (n = 10,000, k = 10; b = 8 as configured, plus the 16/32 fast paths): eigenvalues
    vs the oracle < 1e-10."""
    k = 10
    A = c1_matrix(10000, k)
    n = A.shape[0]
    omega = np.random.default_rng(7).standard_normal((n, b))
    ref = o.RBL_gpu_semantics(A, k, b, omega=omega, qr_mode="posdiag",
                              reorth_mode="cgs" if order == 0 else "mgs")
    D, V, info = rbl.RBL_gpu(A, k, b, omega=omega, reorth_order=order, return_info=True)
    assert ref.converged and info.converged
    assert info.iters == ref.iters
    rel = np.abs(D - ref.D) / np.abs(ref.D)
    assert rel.max() < EIG_TOL, rel
    ov = np.abs(np.sum(V * ref.V, axis=0)) / (np.linalg.norm(V, axis=0) * np.linalg.norm(ref.V, axis=0))
    assert (1 - ov).max() < VEC_TOL, 1 - ov
    res = np.linalg.norm(A @ V - V * D, axis=0) / np.abs(D)
    assert res.max() < RES_TOL, res


@pytest.mark.parametrize("b", [8, 32])
def test_eigenpairs_c1_random_symmetric(rbl, b):
    """C1 exactly as SURVEY §8(d) defines it — A = R + R^T, R at 1 % density with N(0,1)
    values, plus the planted diagonal; n = 10,000, k = 10, b = 8 (and the b = 32 fast paths):
    an unbanded matrix (at this n every 512-row block spans all 40 column panels, so b = 32
    takes the column panels, Q staged whole per block; b = 8 the gather).
    Eigenvalues vs the oracle < 1e-10, the same step count, eigenvectors and residuals."""
    k = 10
    A = matgen.random_sym_csr(10000, 0.01, 20261015, matgen.planted_spectrum(k))
    n = A.shape[0]
    omega = np.random.default_rng(1).standard_normal((n, b))
    ref = o.RBL_gpu_semantics(A, k, b, omega=omega, qr_mode="posdiag")
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        assert ctx.spmm_kernel_for(b) == (7 if b == 32 else 1)
    D, V, info = rbl.RBL_gpu(A, k, b, omega=omega, return_info=True)
    assert ref.converged and info.converged
    assert info.iters == ref.iters
    rel = np.abs(D - ref.D) / np.abs(ref.D)
    assert rel.max() < EIG_TOL, rel
    ov = np.abs(np.sum(V * ref.V, axis=0)) / (np.linalg.norm(V, axis=0) * np.linalg.norm(ref.V, axis=0))
    assert (1 - ov).max() < VEC_TOL, 1 - ov
    res = np.linalg.norm(A @ V - V * D, axis=0) / np.abs(D)
    assert res.max() < RES_TOL, res


@pytest.mark.parametrize("suite", ["moderate", "slow", "step"])
def test_reference_known_answer_suites_on_gpu(rbl, suite):
    """Julia/Unit Testing/*_dec.jl run through the HIP path (the reference only runs them on
    its CPU RBL): relative error norm < 1e-13."""
    gen, ns, k, b = o.KNOWN_ANSWER_SUITES[suite]
    for n in ns:
        A, eig = gen(n, k)
        D, V, info = rbl.RBL_gpu(A, k, b, seed=1000 + n, return_info=True)
        assert info.converged, (suite, n)
        err = np.linalg.norm((D - eig) / eig)
        assert err < o.KNOWN_ANSWER_TOL, (suite, n, err)


def test_known_answer_with_oracle_omega(rbl):
    """Same Omega on both sides: eigenvalues agree with the oracle to 1e-10 on a suite case
    that runs through Krylov exhaustion (n = 100 spans R^n after 20 blocks)."""
    A, eig = o.slow_decay_matrix(100, 5)
    omega = np.random.default_rng(0).standard_normal((100, 5))
    ref = o.RBL_gpu_semantics(A, 5, 5, omega=omega, qr_mode="posdiag", reorth_mode="cgs")
    D, V, info = rbl.RBL_gpu(A, 5, 5, omega=omega, return_info=True)
    assert np.abs(D - ref.D).max() / np.abs(ref.D).max() < EIG_TOL


def test_basis_orthonormal(rbl):
    A = c1_matrix(6000, 10)
    b = 16
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        rbl.lanczos(ctx, 10, b, seed=3, check=False, max_steps=10, ritz=False)
        Q = np.hstack([ctx.get_block(j) for j in range(1, ctx.num_blocks() + 1)])
    G = Q.T @ Q
    assert np.abs(G - np.eye(G.shape[0])).max() < 1e-8


def test_nonconvergence_warning(rbl):
    A, _ = o.slow_decay_matrix(3000, 5)
    D, V, info = rbl.RBL_gpu(A, 5, 5, kryl_sz=60, seed=1, return_info=True)
    assert not info.converged and info.status == 1
    assert V is not None and V.shape == (3000, 5)


def test_zero_and_tiny_matrices(rbl):
    """Edge cases: an all-zero matrix (U == 0: R = 0, Krylov breakdown) and n < b."""
    import scipy.sparse as sp
    Z = sp.csr_matrix((50, 50))
    D, V, info = rbl.RBL_gpu(Z, 2, 4, seed=1, return_info=True)
    assert info.converged and np.all(D == 0)
    A = sp.diags(np.arange(1.0, 13.0)).tocsr()  # n = 12, b = 4: R^n exhausted after 3 blocks
    D, V, info = rbl.RBL_gpu(A, 2, 4, seed=2, return_info=True)
    assert info.converged
    assert np.allclose(D, [12.0, 11.0], rtol=1e-12)


def test_invalid_arguments_fail_loudly(rbl):
    with rbl.Context(0) as ctx:
        with pytest.raises(rbl.RBLError):
            ctx.start(8, 10)                      # no matrix
        ctx.set_matrix(c1_matrix(1000, 2))
        with pytest.raises(rbl.RBLError):
            ctx.start(513, 10)                    # b > RBL_MAX_BLOCK
        ctx.start(8, 4, seed=1)
        with pytest.raises(rbl.RBLError):
            ctx.step(3, False)                    # out of order


def test_stage_timers(rbl):
    A = c1_matrix(5000, 4)
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        ctx.set_option(0, 1)
        rbl.lanczos(ctx, 4, 8, seed=1, check=False, max_steps=8, ritz=True)
        t = ctx.timers()
    for s in ("AQ", "3-term", "qr", "part reorth", "loc reorth"):
        assert t[s] > 0.0, (s, t)


def test_stage_timers_roofline_only(rbl):
    """RBL_OPT_TIMERS 2 (the bench's timed region): events around "AQ" and "part reorth" only;
    other values are refused."""
    from rbl import _lib
    A = c1_matrix(5000, 4)
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        with pytest.raises(rbl.RBLError):
            ctx.set_option(_lib.RBL_OPT_TIMERS, 3)
        ctx.set_option(_lib.RBL_OPT_TIMERS, 2)
        rbl.lanczos(ctx, 4, 8, seed=1, check=False, max_steps=8, ritz=True)
        t = ctx.timers()
    assert t["AQ"] > 0.0 and t["part reorth"] > 0.0, t
    assert all(v == 0.0 for s, v in t.items() if s not in ("AQ", "part reorth")), t


@pytest.mark.parametrize("b,k", [(16, 7), (32, 5)])
def test_ritz_odd_k(rbl, b, k):
    """Ritz projection with an odd number of vectors on the b = 16 / 32 MFMA paths."""
    A = c1_matrix(6000, 10)
    n = A.shape[0]
    omega = np.random.default_rng(5).standard_normal((n, b))
    ref = o.RBL_gpu_semantics(A, k, b, omega=omega, qr_mode="posdiag", reorth_mode="cgs")
    D, V, info = rbl.RBL_gpu(A, k, b, omega=omega, return_info=True)
    assert ref.converged and info.converged and V.shape == (n, k)
    assert np.all(np.abs(D - ref.D) <= EIG_TOL * np.abs(ref.D))
    dots = np.abs(np.sum(V * ref.V, axis=0)) / (np.linalg.norm(V, axis=0) * np.linalg.norm(ref.V, axis=0))
    assert np.all(1 - dots < VEC_TOL), dots
    res = np.linalg.norm(A @ V - V * D[None, :], axis=0) / np.abs(D)
    assert res.max() < RES_TOL


@pytest.mark.parametrize("b", [8, 32])
def test_async_steps_match_sync_steps(rbl, b):
    from rbl import _lib
    """rbl_step_async + rbl_fetch (the host loop's default) against one rbl_step per step: the
    same kernels in the same order, so every A_i, B_{i+1} agrees bit for bit; the stashed
    statuses and the rbl_step / rbl_fetch ordering rules hold."""
    A = c1_matrix(6000, 6)
    steps = 9
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        ctx.start(b, steps, seed=3)
        sync = [ctx.step(i, i >= 2 and i % 2 == 0)[:2] for i in range(1, steps + 1)]
        ctx.start(b, steps, seed=3)
        for i in range(1, 5):
            ctx.step_async(i, i >= 2 and i % 2 == 0)
        with pytest.raises(rbl.RBLError):
            ctx.step(5, False)                    # unfetched asynchronous steps
        with pytest.raises(rbl.RBLError):
            ctx.fetch(2, 4)                       # must start at the first unfetched step
        got = ctx.fetch(1, 3) + ctx.fetch(3, 5)
        for i in range(5, steps + 1):
            ctx.step_async(i, i >= 2 and i % 2 == 0)
        got += ctx.fetch(5, steps + 1)
    assert len(got) == steps
    for (As, Bs), (Aa, Ba, st) in zip(sync, got):
        assert st in (_lib.RBL_OK, _lib.RBL_WARN_QR_SHIFTED)
        assert np.array_equal(As, Aa) and np.array_equal(Bs, Ba)


@pytest.mark.parametrize("b", [80, 128])
def test_block_sizes_past_64(rbl, b):
    """RBL_gpu(A, k, b) takes any b (RBL_gpu.jl:205): b > 64 runs the generic MFMA Gram /
    update kernels with wide panels, the column-blocked gather SpMM and the b x b Cholesky in
    an L2 scratch.  Eigenvalues vs the oracle < 1e-10, residuals < 1e-7."""
    k = 20
    A = c1_matrix(4000, k)
    n = A.shape[0]
    omega = np.random.default_rng(b).standard_normal((n, b))
    ref = o.RBL_gpu_semantics(A, k, b, omega=omega, qr_mode="posdiag", reorth_mode="cgs")
    D, V, info = rbl.RBL_gpu(A, k, b, omega=omega, return_info=True)
    assert ref.converged and info.converged and info.iters == ref.iters
    rel = np.abs(D - ref.D) / np.abs(ref.D)
    assert rel.max() < EIG_TOL, rel
    res = np.linalg.norm(A @ V - V * D, axis=0) / np.abs(D)
    assert res.max() < RES_TOL, res
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        X = np.random.default_rng(3).standard_normal((n, b))
        Y = ctx.apply(X)
    ref_y = A @ X
    assert np.abs(Y - ref_y).max() <= 1e-12 * np.abs(ref_y).max()


def test_dense_block_size_past_64(rbl):
    """Dense A with b = 96: the gathered-Q buffer is re-sized past its 64-column default.
    (n stays above the Krylov dimension at the first convergence check: once a block only
    partly fits in R^n, the reference's own answer carries spurious Ritz values that depend
    on its QR's junk columns — DESIGN §4, not a parity case.)"""
    n, k, b = 2000, 6, 96
    rng = np.random.default_rng(2)
    B = rng.standard_normal((n, n)) / np.sqrt(n)
    A = B + B.T + np.diag(np.r_[np.linspace(40, 30, 2 * k), np.zeros(n - 2 * k)])
    omega = rng.standard_normal((n, b))
    ref = o.RBL_gpu_semantics(A, k, b, omega=omega, qr_mode="posdiag", reorth_mode="cgs")
    D, V, info = rbl.RBL_gpu(A, k, b, omega=omega, return_info=True)
    assert ref.converged and info.converged
    assert (np.abs(D - ref.D) / np.abs(ref.D)).max() < EIG_TOL


@pytest.mark.parametrize("b,bits", [(16, 64), (32, 64), (32, 32)])
def test_pass_fusions(rbl, b, bits):
    """RBL_OPT_FUSE: the 3-pass CholQR2 (bit 0) gives the same bits as the 4-pass form; the
    local-reorth Gram formed inside the QR (bit 1) agrees to rounding (1e-12 relative) —
    over 12 steps of the C1-like matrix, per-step A_i and B_{i+1}."""
    from rbl import _lib
    A = c1_matrix(4000, 10)
    n = A.shape[0]
    omega = np.random.default_rng(b).standard_normal((n, b))
    out = {}
    for fuse in (0, 1, 3):
        with rbl.Context(0) as ctx:
            ctx.set_option(_lib.RBL_OPT_FUSE, fuse)
            ctx.set_matrix(A)
            _, _, info = rbl.lanczos(ctx, 10, b, omega=omega, check=False, max_steps=12,
                                     trace=True, ritz=False, basis_bits=bits)
        out[fuse] = (np.array(info.trace_A), np.array(info.trace_B))
    assert np.array_equal(out[0][0], out[1][0]) and np.array_equal(out[0][1], out[1][1])
    for t in (0, 1):
        d = np.abs(out[3][t] - out[1][t]).max() / np.abs(out[1][t]).max()
        assert d < 1e-12, (t, d)


@pytest.mark.parametrize("n,W", [(4000, 64), (40003, 64), (100003, 64), (50001, 32)])
def test_local_reorth_fused_into_spmm(rbl, n, W):
    """RBL_OPT_FUSE bit 2: the local reorth Q_i -= Q_{i-1} C (RBL_gpu.jl:83-93) applied by the
    band-tile SpMM as it stages Q_i's rows — interior rows written back by the SpMM, the first
    and last H rows of every workgroup range by k_locfix afterwards.  n covers ranges shorter
    than 2H (all rows by k_locfix), just over it, long ones, H = 32 and a ragged last tile.
    Per-step A_i / B_{i+1} and the Ritz pairs agree with the separate pass (fuse 3) to 1e-12."""
    from rbl import _lib
    k, b = 10, 32
    plant = matgen.planted_spectrum(k)
    omega = np.random.default_rng(n).standard_normal((n, b))
    out = {}
    for fuse in (3, 7):
        with rbl.Context(0) as ctx:
            ctx.set_option(_lib.RBL_OPT_FUSE, fuse)
            ctx.gen_hashwindow(n, W, 0.7734, 11, plant)
            assert ctx.spmm_kernel_for(b) == 5  # band tiles: the fused path applies
            D, V, info = rbl.lanczos(ctx, k, b, omega=omega, trace=True)
        assert info.converged
        out[fuse] = (np.array(info.trace_A), np.array(info.trace_B), D, V)

    assert out[3][0].shape == out[7][0].shape
    for t in (0, 1):
        d = np.abs(out[7][t] - out[3][t]).max() / np.abs(out[3][t]).max()
        assert d < 1e-12, (t, d)
    D3, V3, D7, V7 = out[3][2], out[3][3], out[7][2], out[7][3]
    assert (np.abs(D7 - D3) / np.abs(D3)).max() < 1e-12
    assert (1 - np.abs(np.sum(V7 * V3, axis=0))).max() < 1e-10


@pytest.mark.parametrize("case", ["converges", "runs_out"])
def test_speculative_steps_change_nothing(rbl, case):
    """Steps enqueued ahead of a convergence check (rbl.lanczos speculate) leave D, V, the step
    count and every A_i / B_{i+1} bit for bit as in the strict alternation (reference order):
    a run converging at a check (the extra steps are discarded) and one using all its steps."""
    k, b = 10, 16
    if case == "converges":
        A = c1_matrix(4000, k)
    else:
        A, _ = o.slow_decay_matrix(3000, k)
        A = (A + matgen.hashwindow_csr(3000, 8, 0.5, 3, None) * 1e-3).tocsr()
    omega = np.random.default_rng(5).standard_normal((A.shape[0], b))
    out = []
    for spec in (False, 3, "auto"):
        with rbl.Context(0) as ctx:
            ctx.set_matrix(A)
            D, V, info = rbl.lanczos(ctx, k, b, omega=omega, trace=True, speculate=spec)
        out.append((D, V, info))
    D0, V0, i0 = out[0]
    assert i0.spec_steps == 0 and out[1][2].spec_steps > 0
    if case == "runs_out":   # residuals far above the tolerance: "auto" runs ahead from check 3 on
        assert out[2][2].spec_steps > 0 and out[2][2].spec_wasted == 0
    for D1, V1, i1 in out[1:]:
        assert i0.iters == i1.iters and i0.converged == i1.converged
        assert np.array_equal(D0, D1) and np.array_equal(V0, V1)
        assert all(np.array_equal(a, c) for a, c in zip(i0.trace_A, i1.trace_A))
        assert all(np.array_equal(a, c) for a, c in zip(i0.trace_B, i1.trace_B))


@pytest.mark.parametrize("b", [16, 32])
def test_local_reorth_gram_after_shifted_third_pass(rbl, monkeypatch, b):
    """The next step's local-reorth Gram formed inside the QR (RBL_OPT_FUSE bit 1) when CholQR
    takes its shifted third pass: Z^T Q3 = (Z^T Q2) R3^-1 (k_cloc_rinv), the partials of Z^T Q2
    all-reduced with the pass-3 Gram.  A diagonal A of rank 4.5 b: the block Krylov space is
    range(A) (Q_1 = qr(A Omega)), so step 4's U has b/2 directions above rounding and its QR is
    shifted (an even step: the next one runs no partial reorth, so the Gram rides on this QR);
    step 5's local reorth then removes the new block's (rounding-born) Q_4 components with it.  After 5 steps ||Q_4^T Q_5|| is at rounding (1e-12) with the Gram fused (3)
    and separate (1); without the R3^-1 factor (RBL_DIAG_CLOC_NOFIX, the negative control) it is
    not, so the test sees the factor."""
    import scipy.sparse as sp
    from rbl import _lib
    n, D = 2000, 9 * b // 2
    lam = np.zeros(n)
    lam[:D] = np.linspace(1.0, 10.0, D)
    A = sp.diags(lam).tocsc()
    omega = np.random.default_rng(b).standard_normal((n, b))

    def run(fuse):
        with rbl.Context(0) as ctx:
            ctx.set_option(_lib.RBL_OPT_FUSE, fuse)
            ctx.set_matrix(A)
            ctx.start(b, 8, omega=omega)
            for i in range(1, 6):
                ctx.step_async(i, i >= 2 and i % 2 == 0)
            st = [s for _, _, s in ctx.fetch(1, 6)]
            Q4, Q5 = ctx.get_block(4), ctx.get_block(5)
        return st, np.abs(Q4.T @ Q5).max()

    st3, e3 = run(3)
    st1, e1 = run(1)
    monkeypatch.setenv("RBL_DIAG_CLOC_NOFIX", "1")
    st3n, e3n = run(3)
    print(f"b={b}: statuses {st3} / {st1}; |Q4^T Q5| fused {e3:.2e}, separate {e1:.2e}, "
          f"fused without R3^-1 {e3n:.2e}")
    assert st3[3] == _lib.RBL_WARN_QR_SHIFTED and st1[3] == _lib.RBL_WARN_QR_SHIFTED
    assert e3 < 1e-12 and e1 < 1e-12
    assert e3n > 1e3 * e3



@pytest.mark.parametrize("b", [16, 32])
def test_cholqr_default_kernel_known_answers(rbl, b):
    """The product's CholQR small part (k_chol_elim2 at b = 16 / 32: R^-1 formed in the
    factorisation's own sweep) on the reference's known-answer suites (moderate and slow decay,
    n = 300, k = 5) within the suites' 1e-13 (test.jl:16-50), and through Krylov exhaustion (the
    slow-decay matrix at n = 9 b: the last step factors a numerically zero block, the shifted /
    zero paths) with finite A_i / B_{i+1}.  Its bit identity with the other Cholesky
    kernels is a variants-build test (test_gpu_variants)."""
    for gen in (o.moderate_decay_matrix, o.slow_decay_matrix):
        A, eig = gen(300, 5)
        D, V, info = rbl.RBL_gpu(A, 5, b, seed=3, return_info=True)
        assert info.converged and np.linalg.norm((D - eig) / eig) < o.KNOWN_ANSWER_TOL
    A, _ = o.slow_decay_matrix(9 * b, 5)
    omega = np.random.default_rng(b).standard_normal((9 * b, b))
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        _, _, info = rbl.lanczos(ctx, 5, b, omega=omega, check=False, max_steps=9, trace=True,
                                 ritz=False)
    assert len(info.trace_A) == 9
    assert all(np.all(np.isfinite(t)) for t in info.trace_A + info.trace_B)


@pytest.mark.parametrize("bits", [64, 32])
def test_ritz_row_pieces(rbl, bits):
    """rbl_ritz at a size where its row-piece form applies (n_local x k x 8 B >= 256 MiB: the
    combination V = [Q] S in 8 row pieces on a side stream with the staged D2H behind them;
    RBL_gpu.jl:106-132 / :219) takes that path (rbl_path_stats' ritz_pieces), returns Ritz
    pairs with residual ||A v - lambda v|| / |lambda| < 1e-7 and orthonormal vectors to 1e-9
    (1e-5 and 1e-6 with the fp32 basis), and two more runs on the same context return the same D and V bit for
    bit (the side stream's use of the run scratch is ordered before the next run's steps)."""
    import scipy.sparse as sp
    n, b, k = 2_000_000, 32, 20
    out = []
    with rbl.Context(0) as ctx:
        ctx.gen_hashwindow(n, 64, 0.7734, 5, matgen.planted_spectrum(k))
        rowptr, col, val = ctx.get_matrix_csr()
        A = sp.csr_matrix((val, col, rowptr.astype(np.int32)), shape=(n, n))
        for _ in range(3):
            ctx.path_stats(reset=True)
            D, V, info = rbl.lanczos(ctx, k, b, seed=2, basis_bits=bits)
            assert info.converged and ctx.path_stats()["ritz_pieces"] == 1
            out.append((D, V))
    D0, V0 = out[0]
    res = np.linalg.norm(A @ V0 - V0 * D0, axis=0) / np.abs(D0)
    assert res.max() < (RES_TOL if bits == 64 else 1e-5), res
    assert np.abs(V0.T @ V0 - np.eye(k)).max() < (1e-9 if bits == 64 else 1e-6)
    for D1, V1 in out[1:]:
        assert np.array_equal(D0, D1) and np.array_equal(V0, V1)
