"""GPU: the measured-and-rejected kernel variants and A/B switches of the VARIANTS build.

The product library (librbl_hip.so built by csrc/Makefile) leaves these out: two waves per SIMD
in the band-tile SpMM (RBL_BT2), packed and half band tiles (RBL_BT_PACK / RBL_BT_HALF), the
degree-ranked column tiers of one rank (RBL_SEG_TIERS), the fp32 local reorth on the MFMA tile
kernels (RBL_LOC32_MFMA), the other Cholesky kernels (RBL_CHOL_REG), the earlier reductions and
stash (RBL_RED_CHUNK, RBL_REDUCE_NARROW, RBL_STASH_COPY) and the one-pass Ritz
(RBL_RITZ_SERIAL, with RBL_RITZ_TRACE).  DESIGN.md records why each was measured and kept off.
They are built for diagnostics only:

    bash tools/build_variant.sh variants "-DRBL_VARIANTS"
    RBL_LIB=tools/variants/variants/librbl_hip.so python -m pytest tests/test_gpu_variants.py -m gpu

This module is skipped against the product library (rbl._lib.VARIANTS false).  Each test
checks that its variant gives the product path's results (bit for bit where the arithmetic is
the same, else to the stated tolerance).
"""
import numpy as np
import pytest
import scipy.sparse as sp

from oracle import matgen
from oracle import rbl_oracle as o
from test_gpu_multirank import run_ranks


def _variants_built():
    try:
        from rbl import _lib
        return _lib.VARIANTS
    except Exception:  # noqa: BLE001 — no library: the GPU suite fails elsewhere, loudly
        return False


pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not _variants_built(),
                                 reason="product library: the variants are built only by "
                                        "tools/build_variant.sh with -DRBL_VARIANTS")]


CASE = dict(n=6000, scale=13, edges=120_000, seed=7)   # test_gpu_rmat's R-MAT case
STEP_TOL = 2e-6  # x ||A||_1, absolute (test_gpu_fp32_basis)


@pytest.fixture(scope="module")
def rbl():
    import rbl as _r
    return _r


def c1_matrix(n=10000, k=10, W=64, seed=20261015):
    """symmetric hash-window + planted top spectrum."""
    p = min(1.0, 0.01 * n / (2 * W)) if n <= 2 * W * 100 else 0.7734
    return matgen.hashwindow_csr(n, W, p, seed, matgen.planted_spectrum(k))


def _check(A, Y, X):
    ref = A @ X
    bound = (abs(A) @ np.abs(X)) * 1e-13 + 1e-300
    assert np.all(np.abs(Y - ref) <= bound), np.max(np.abs(Y - ref) / bound)


@pytest.mark.parametrize("b", [16, 32])
@pytest.mark.parametrize("n,W,p", [(7000, 64, 0.7734), (5003, 30, 0.9), (300, 60, 1.0), (100, 30, 0.95)])
def test_spmm_band_tiles_packed_bit_identical(rbl, monkeypatch, n, W, p, b):
    """Packed band tiles (zeros dropped, RBL_BT_PACK=1) against the dense tiles (the
    default): the MFMA operands are the same values, so U and every Lanczos block A_i
    (fused epilogue + A_i partials) must agree bit for bit."""
    A = matgen.hashwindow_csr(n, W, p, n + 11)
    X = np.random.default_rng(n + 1).standard_normal((n, b))
    out = []
    monkeypatch.setenv("RBL_BT2", "0")  # packed tiles run k_spmm_bt only: compare like with like
    for pack in ("0", "1"):
        monkeypatch.setenv("RBL_BT_PACK", pack)
        with rbl.Context(0) as ctx:
            ctx.set_matrix(A)
            assert ctx.spmm_kernel_for(b) == 5
            Y = ctx.apply(X)
            _, _, info = rbl.lanczos(ctx, 4, b, seed=2, check=False, max_steps=4, trace=True,
                                     ritz=False)
        out.append((Y, info.trace_A))
    _check(A, out[1][0], X)
    assert np.array_equal(out[0][0], out[1][0])
    for a0, a1 in zip(out[0][1], out[1][1]):
        assert np.array_equal(a0, a1)


@pytest.mark.parametrize("n,W,b,bits", [(50003, 64, 32, 64), (20001, 32, 32, 64),
                                         (30000, 64, 16, 64), (12345, 32, 16, 64),
                                         (40000, 64, 32, 32), (300, 32, 16, 64)])
def test_spmm_half_band_tiles_bit_identical(rbl, monkeypatch, n, W, b, bits):
    """Half band tiles (A symmetric: diagonal block + right strip stored, the left groups
    transposed back in the kernel from the previous tiles' strips) against the whole tiles
    (RBL_BT_HALF=0): the MFMA operands are the same values in the same order, so U, every
    Lanczos A_i / B_{i+1} (fused epilogue, A_i partials, fused local reorth, fp32 basis) and
    the Ritz pairs agree bit for bit.  n = 300: a single workgroup range."""
    plant = matgen.planted_spectrum(5)
    A = matgen.hashwindow_csr(n, W, 0.7734, n + 5, plant)
    X = np.random.default_rng(n + 2).standard_normal((n, b))
    out = []
    for half in ("0", "1"):
        monkeypatch.setenv("RBL_BT_HALF", half)  # opt-in format
        with rbl.Context(0) as ctx:
            ctx.set_matrix(A)
            assert ctx.spmm_kernel_for(b) == 5
            assert ctx.matrix_format() == (3 if half == "1" else 1)
            Y = ctx.apply(X)
            D, V, info = rbl.lanczos(ctx, 5, b, seed=2, check=False, max_steps=min(8, n // b),
                                     trace=True, basis_bits=bits)
        out.append((Y, info, D, V))
    _check(A, out[1][0], X)
    assert np.array_equal(out[0][0], out[1][0])
    for a0, a1 in zip(out[0][1].trace_A + out[0][1].trace_B, out[1][1].trace_A + out[1][1].trace_B):
        assert np.array_equal(a0, a1)
    assert np.array_equal(out[0][2], out[1][2]) and np.array_equal(out[0][3], out[1][3])


def test_spmm_half_band_tiles_need_exact_symmetry(rbl, monkeypatch):
    """One nonzero whose mirror differs in the last bit keeps the whole tiles (format 1)."""
    monkeypatch.setenv("RBL_BT_HALF", "1")
    A = matgen.hashwindow_csr(5000, 64, 0.7734, 3).tolil()
    A[100, 140] = np.nextafter(A[140, 100], np.inf) if A[140, 100] != 0 else 1.0
    A = sp.csr_matrix(A)
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        assert ctx.spmm_kernel_for(32) == 5 and ctx.matrix_format() == 1
        X = np.random.default_rng(0).standard_normal((5000, 32))
        _check(A, ctx.apply(X), X)


@pytest.mark.parametrize("n,W,half,fuse", [(50003, 64, "0", 7), (50003, 64, "1", 7), (20001, 32, "0", 7),
                                           (20001, 32, "1", 3), (300, 64, "0", 7), (4099, 64, "1", 3)])
def test_spmm_band_tiles_two_waves_per_simd(rbl, monkeypatch, n, W, half, fuse):
    """k_spmm_bt2 (RBL_BT2=1: eight waves share the Q ring, waves p and p + 4 of a SIMD split a
    tile's band groups) against k_spmm_bt: the same products, the group sum associated as (left
    groups) + (the rest), so per-step A_i / B_{i+1} agree to 1e-12 relative over a 10-step
    Lanczos run (fused 3-term epilogue, A_i partials, with and without the fused local
    reorth); whole and half tiles; H = 32 and 64; a matrix smaller than one round (its run kept
    well short of Krylov exhaustion, where the trace amplifies rounding)."""
    plant = matgen.planted_spectrum(5)
    A = matgen.hashwindow_csr(n, W, 0.7734, n + 9, plant)
    monkeypatch.setenv("RBL_BT_HALF", half)
    runs = []
    for v in ("0", "1"):
        monkeypatch.setenv("RBL_BT2", v)
        with rbl.Context(0) as ctx:
            ctx.set_option(rbl._lib.RBL_OPT_FUSE, fuse)
            ctx.set_matrix(A)
            assert ctx.spmm_kernel_for(32) == 5
            _, _, info = rbl.lanczos(ctx, 5, 32, seed=4, check=False, max_steps=min(10, n // 64),
                                     trace=True, ritz=False)
        runs.append(info)
    for a0, a1 in zip(runs[0].trace_A + runs[0].trace_B, runs[1].trace_A + runs[1].trace_B):
        assert np.abs(a0 - a1).max() <= 1e-12 * np.abs(a0).max()


@pytest.mark.parametrize("bt2", ["1"])
@pytest.mark.parametrize("P", [1, 2])
def test_variants_fused_local_reorth_runs_two_waves(rbl, monkeypatch, P, bt2):
    """The fused path really replaces the separate pass on 1 and 2 ranks, with the one-wave
    band-tile SpMM (RBL_BT2=0, default) and the two-waves-per-SIMD one (RBL_BT2=1).  Asserted on
    the library's path counters (rbl_path_stats), not on stage times: with both ranks on one GPU
    a stage's events also span the other rank's kernels (round 4's RBL_BT2=1 run measured rank
    0's loc-reorth stage at 2.65 ms fused against 1.46 ms separate — about one of rank 1's SpMM
    launches per step, ~0.37 ms at 1e6 rows, waiting in front of rank 0's small fix-up kernels
    while the persistent SpMM held every CU's LDS).  Fused (RBL_OPT_FUSE 7): every step from
    i = 2 on applies the update inside the SpMM, fixes the range edges after it (and on several
    ranks the rank edges before the exchange), and runs no separate pass; unfused (3): a
    separate pass per step and no fused SpMM.  Both give the same A_i / B_{i+1} to 1e-12."""
    monkeypatch.setenv("RBL_BT2", bt2)
    n, W, k, b, steps = 2_000_000, 64, 10, 32, 8
    plant = matgen.planted_spectrum(k)

    def run(fuse):
        def fn(ctx, r):
            ctx.set_option(rbl._lib.RBL_OPT_FUSE, fuse)
            ctx.gen_hashwindow(n, W, 0.7734, 17, plant)
            assert ctx.spmm_kernel_for(b) == 5
            ctx.path_stats(reset=True)
            _, _, info = rbl.lanczos(ctx, k, b, seed=9, check=False, max_steps=steps,
                                     ritz=False, trace=True)
            return ctx.path_stats(), info
        if P == 1:
            with rbl.Context(0) as ctx:
                return [fn(ctx, 0)]
        return run_ranks(rbl, P, fn)

    t7, t3 = run(7), run(3)
    for (p7, i7), (p3, i3) in zip(t7, t3):
        loc_steps = len(i7.trace_A) - 1                    # block steps i >= 2
        assert loc_steps >= 6 and p7["spmm"] == p3["spmm"] == len(i7.trace_A) + 1
        assert p7["spmm_loc_fused"] == loc_steps and p7["loc_separate"] == 0
        assert p7["locfix_rest"] == loc_steps
        assert p7["locfix_edges"] == (loc_steps if P > 1 else 0)
        assert p3["spmm_loc_fused"] == 0 and p3["loc_separate"] == loc_steps
        assert p3["locfix_rest"] == p3["locfix_edges"] == 0
        if bt2 == "1":   # every step launch (EPI + A_i partials) on the two-wave kernel
            assert p7["spmm_two_wave"] >= loc_steps and p3["spmm_two_wave"] >= loc_steps
        else:
            assert p7["spmm_two_wave"] == p3["spmm_two_wave"] == 0
        for a, a1 in zip(i7.trace_A + i7.trace_B, i3.trace_A + i3.trace_B):
            assert np.abs(a - a1).max() <= 1e-12 * np.abs(a1).max()


def test_multirank_half_band_tiles_bit_identical(rbl, monkeypatch):
    """Half band tiles on 3 ranks (each rank's first NGL tiles whole, their left groups reach
    into the previous rank's rows) against whole tiles: A_i / B_{i+1} bit for bit."""
    n, W, p, seed, k, b = 30001, 64, 0.7734, 23, 10, 32
    plant = matgen.planted_spectrum(k)

    def run(half):
        monkeypatch.setenv("RBL_BT_HALF", half)

        def fn(ctx, r):
            ctx.gen_hashwindow(n, W, p, seed, plant)
            assert ctx.matrix_format() == (3 if half == "1" else 1)
            _, _, info = rbl.lanczos(ctx, k, b, seed=3, check=False, max_steps=10, trace=True,
                                     ritz=False)
            return info
        return run_ranks(rbl, 3, fn)

    h, w = run("1"), run("0")
    for ih, iw in zip(h, w):
        for a, a1 in zip(ih.trace_A + ih.trace_B, iw.trace_A + iw.trace_B):
            assert np.array_equal(a, a1)


@pytest.mark.parametrize("dense", [False, True])
def test_fp32_local_reorth_row_kernel_matches_tile_kernel(rbl, dense, monkeypatch):
    """b = 32: the fp32 local reorth runs its Gram on four waves per split (k_gram32_one) and
    its update as a row-streaming kernel (k_upd32_rows, k_tsmm32's MFMA k order);
    RBL_LOC32_MFMA=1 restores both tile kernels.  Traces and every basis block agree to fp32
    rounding (the Gram's per-split sum order differs)."""
    b, steps = 32, 8
    A = (matgen.hashwindow_csr(6000, 64, 0.7734, 7, matgen.planted_spectrum(10)) if dense
         else c1_matrix(5000, 10))
    n = A.shape[0]
    omega = np.random.default_rng(11).standard_normal((n, b))
    out = []
    for tile in (False, True):
        if tile:
            monkeypatch.setenv("RBL_LOC32_MFMA", "1")
        else:
            monkeypatch.delenv("RBL_LOC32_MFMA", raising=False)
        with rbl.Context(0) as ctx:
            ctx.set_matrix(A)
            _, _, info = rbl.lanczos(ctx, 10, b, omega=omega, check=False, max_steps=steps,
                                     trace=True, ritz=False, basis_bits=32)
            out.append((info, [ctx.get_block(j) for j in range(1, steps + 1)]))
    anorm = abs(A).sum(axis=0).max()
    (i1, q1), (i2, q2) = out
    for a1, a2 in zip(i1.trace_A + i1.trace_B, i2.trace_A + i2.trace_B):
        assert np.abs(a1 - a2).max() <= STEP_TOL * anorm
    for x, y in zip(q1, q2):
        assert np.abs(x - y).max() <= 1e-5
    print("bit-identical blocks:", sum(np.array_equal(x, y) for x, y in zip(q1, q2)), "of", steps)


@pytest.mark.parametrize("tiers", ["64", "64,1024"])
def test_rmat_column_tiers(rbl, tiers, monkeypatch):
    """Column-tiered segmented gather (RBL_SEG_TIERS: the highest-degree columns swept first,
    each tier its own CSR + task table, accumulated into U): the SpMM within 1e-13 |A||X| of
    SciPy, and a fixed-step Lanczos trace equal to the one-sweep kernel's to 1e-12 (only each
    row's sum order differs)."""
    A = matgen.rmat_csr(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"],
                        matgen.planted_spectrum(5))
    X = np.random.default_rng(11).standard_normal((A.shape[0], 32))
    infos = []
    for env in (None, tiers):
        if env is None:
            monkeypatch.delenv("RBL_SEG_TIERS", raising=False)
        else:
            monkeypatch.setenv("RBL_SEG_TIERS", env)
        with rbl.Context(0) as ctx:
            ctx.gen_rmat(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"],
                         matgen.planted_spectrum(5))
            Y = ctx.apply(X)
            _, _, info = rbl.lanczos(ctx, 5, 32, seed=9, check=False, max_steps=8, trace=True,
                                     ritz=False)
            infos.append(info)
        bound = (abs(A) @ np.abs(X)) * 1e-13 + 1e-300
        assert np.all(np.abs(Y - A @ X) <= bound)
    for a0, a1 in zip(infos[0].trace_A, infos[1].trace_A):
        assert np.abs(a0 - a1).max() <= 1e-12 * np.abs(a0).max()


@pytest.mark.parametrize("b,bits", [(16, 64), (32, 64), (32, 32)])
def test_cholqr_register_kernel_bit_identical(rbl, monkeypatch, b, bits):
    """The one-wave register Cholesky (k_chol_reg, b = 16 / 32) against the four-wave LDS kernel
    (RBL_CHOL_REG=0): the same R, R^-1 and Rtot, so 12-step A_i / B_{i+1} traces are bit-identical
    — on the C1-like matrix and through Krylov exhaustion (the reference's slow-decay matrix at
    n = 9 b: the last step factors a numerically zero block, the shifted / zero paths)."""
    A1 = c1_matrix(4000, 10)
    A2, _ = o.slow_decay_matrix(9 * b, 5)
    for A, steps in ((A1, 12), (A2, 9)):
        n = A.shape[0]
        omega = np.random.default_rng(b).standard_normal((n, b))
        out = {}
        for reg in ("0", "1"):
            monkeypatch.setenv("RBL_CHOL_REG", reg)
            with rbl.Context(0) as ctx:
                ctx.set_matrix(A)
                _, _, info = rbl.lanczos(ctx, 5, b, omega=omega, check=False, max_steps=steps,
                                         trace=True, ritz=False, basis_bits=bits)
            out[reg] = (np.array(info.trace_A), np.array(info.trace_B))
        assert np.array_equal(out["0"][0], out["1"][0]) and np.array_equal(out["0"][1], out["1"][1])


@pytest.mark.parametrize("b,bits", [(16, 64), (32, 64), (32, 32)])
def test_cholqr_elimination_kernel(rbl, monkeypatch, b, bits):
    """The one-wave Cholesky that forms R^-1 in the factorisation's own sweep (k_chol_elim2, the
    default RBL_CHOL_REG=2): R and Rtot as the other kernels, R^-1 by forward elimination instead
    of back substitution — 12-step A_i / B_{i+1} traces within 1e-12 of the four-wave kernel's on
    the C1-like matrix and through Krylov exhaustion, and the reference's known-answer suites on
    it (b = 16 / 32: moderate and slow decay at n = 300, k = 5) within the suites' 1e-13.  The
    form on both halves of the wave (2) and on one half (k_chol_elim, 3): the same bits."""
    A1 = c1_matrix(4000, 10)
    A2, _ = o.slow_decay_matrix(9 * b, 5)
    for A, steps in ((A1, 12), (A2, 9)):
        n = A.shape[0]
        omega = np.random.default_rng(b).standard_normal((n, b))
        out = {}
        for reg in ("0", "2", "3"):
            monkeypatch.setenv("RBL_CHOL_REG", reg)
            with rbl.Context(0) as ctx:
                ctx.set_matrix(A)
                _, _, info = rbl.lanczos(ctx, 5, b, omega=omega, check=False, max_steps=steps,
                                         trace=True, ritz=False, basis_bits=bits)
            out[reg] = (np.array(info.trace_A), np.array(info.trace_B))
        assert np.array_equal(out["2"][0], out["3"][0]) and np.array_equal(out["2"][1], out["3"][1])
        for t in (0, 1):
            scale = np.abs(out["0"][t]).max()
            d = np.abs(out["2"][t] - out["0"][t]).max() / scale
            assert d < 1e-12, (t, d)
    if bits == 64:
        monkeypatch.setenv("RBL_CHOL_REG", "2")
        for gen in (o.moderate_decay_matrix, o.slow_decay_matrix):
            A, eig = gen(300, 5)
            D, V, info = rbl.RBL_gpu(A, 5, b, seed=3, return_info=True)
            assert info.converged and np.linalg.norm((D - eig) / eig) < o.KNOWN_ANSWER_TOL


def test_latency_knobs_agree(rbl, monkeypatch):
    """The A/B switches of round 5's latency work: RBL_STASH_COPY=1 (a device record and one D2H
    copy instead of k_stash writing pinned memory) gives the same bits; RBL_REDUCE_NARROW=1 and
    RBL_RED_CHUNK=0 (the earlier Gram-partial reductions: other summation trees) the same A_i /
    B_{i+1} to 1e-12 — at n = 40,000, where the b x b Grams have > 64 partials (k_reduce_wide) and
    the update's local-reorth Gram one per 128 rows (chunked levels)."""
    A = c1_matrix(40000, 10)
    b = 32
    omega = np.random.default_rng(4).standard_normal((A.shape[0], b))

    def run():
        with rbl.Context(0) as ctx:
            ctx.set_matrix(A)
            _, _, info = rbl.lanczos(ctx, 10, b, omega=omega, check=False, max_steps=12,
                                     trace=True, ritz=False)
        return np.array(info.trace_A), np.array(info.trace_B)

    ref = run()
    for knob, exact in (("RBL_STASH_COPY", True), ("RBL_REDUCE_NARROW", False), ("RBL_RED_CHUNK", False)):
        monkeypatch.setenv(knob, "0" if knob == "RBL_RED_CHUNK" else "1")
        out = run()
        monkeypatch.delenv(knob)
        for t in (0, 1):
            if exact:
                assert np.array_equal(out[t], ref[t]), knob
            else:
                d = np.abs(out[t] - ref[t]).max() / np.abs(ref[t]).max()
                assert d < 1e-12, (knob, t, d)


@pytest.mark.parametrize("bits", [64, 32])
def test_ritz_pipelined_matches_one_pass(rbl, monkeypatch, capfd, bits):
    """rbl_ritz's pipelined form (the combination in 8 row pieces on a side stream, the staged D2H
    behind them on the context's stream; RBL_gpu.jl:106-132 / :219) returns the one-pass form's
    V bit for bit, at a size where it applies (n_local x k x 8 B >= 256 MiB), and takes that path
    (RBL_RITZ_TRACE); a second run on the same context then gives the same D and V again (the side
    stream's use of the run scratch is ordered before the next run's steps).  Both bases: fp64, and
    the fp32 Krylov basis (FLOAT = Float32) whose combination widens on load."""
    n, b, k = 2_000_000, 32, 20
    monkeypatch.setenv("RBL_RITZ_TRACE", "1")
    out = []
    with rbl.Context(0) as ctx:
        ctx.gen_hashwindow(n, 64, 0.7734, 5, matgen.planted_spectrum(k))
        for serial in ("1", None, None):
            if serial:
                monkeypatch.setenv("RBL_RITZ_SERIAL", serial)
            else:
                monkeypatch.delenv("RBL_RITZ_SERIAL", raising=False)
            capfd.readouterr()
            D, V, info = rbl.lanczos(ctx, k, b, seed=2, basis_bits=bits)
            err = capfd.readouterr().err
            assert info.converged and ("pipelined" in err) == (serial is None), err
            out.append((D, V))
    (D0, V0) = out[0]
    for D1, V1 in out[1:]:
        assert V1.shape == (n, k) and np.array_equal(D0, D1)
        assert np.array_equal(V0, V1), np.abs(V0 - V1).max()
