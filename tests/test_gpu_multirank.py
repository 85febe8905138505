"""GPU: the row-partitioned multi-rank path on one GPU.

Ranks are contexts of one in-process LocalGroup, each driven by its own thread; the library
code they run (nnz-balanced partition, halo tables, halo exchange before every SpMM,
distributed Grams + sums, distributed CholQR, Ritz rows) is the code the RCCL transport runs,
only the transport differs (comm.hpp).  RCCL rejects two ranks on one device, so the RCCL
transport is exercised here at one rank only (test_rccl_transport_selftest).

Tolerances: eigenvalues |dλ|/|λ| < 1e-10 against the single-rank run and the oracle (the
partitioned sums only reorder fp64 additions); per-step A_i within 1e-9 relative; Ritz
vectors 1 - |v·v'| < 1e-8.
"""
import threading

import numpy as np
import pytest

from oracle import matgen
from oracle import rbl_oracle as o

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rbl():
    import rbl as _r
    return _r


def run_ranks(rbl, P, fn, timeout=240):
    """Run fn(ctx, rank) on P in-process ranks (one thread each); return the per-rank results."""
    group = rbl.LocalGroup(P)
    out = [None] * P
    errs = []

    def worker(r):
        try:
            with rbl.Context(0, group=group, rank=r) as ctx:
                out[r] = fn(ctx, r)
        except BaseException as e:  # noqa: BLE001 - reported below
            errs.append((r, repr(e)))

    ths = [threading.Thread(target=worker, args=(r,)) for r in range(P)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout)
    group.close()
    assert not any(t.is_alive() for t in ths), "a rank hung"
    assert not errs, errs
    return out


def _single(rbl, A, k, b, omega, steps=None, check=True):
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        return rbl.lanczos(ctx, k, b, omega=omega, check=check, max_steps=steps, trace=True)


@pytest.mark.parametrize("P", [2, 3, 4])
def test_multirank_apply_matches_scipy(rbl, P):
    A = matgen.hashwindow_csr(5000, 40, 0.6, 3, matgen.planted_spectrum(5))
    X = np.random.default_rng(P).standard_normal((A.shape[0], 16))

    def fn(ctx, r):
        ctx.set_matrix(A)
        n, r0, r1, _ = ctx.matrix_info()
        return r0, r1, ctx.apply(X[r0:r1])

    parts = run_ranks(rbl, P, fn)
    assert parts[0][0] == 0 and parts[-1][1] == A.shape[0]
    for (a0, a1, _), (b0, _, _) in zip(parts, parts[1:]):
        assert a1 == b0
    Y = np.vstack([y for _, _, y in parts])
    ref = A @ X
    assert np.abs(Y - ref).max() <= 1e-12 * np.abs(ref).max()


@pytest.mark.parametrize("P", [2, 3])
def test_multirank_column_panels(rbl, P):
    """The column-panel SpMM on P ranks (range halo of W = 600 rows per side): rbl_apply equals
    SciPy to 1e-12, and 6 block steps equal the single rank's A_i / B_{i+1} to 1e-10."""
    A = matgen.hashwindow_csr(20000, 600, 0.08, 21, matgen.planted_spectrum(5))
    X = np.random.default_rng(P).standard_normal((A.shape[0], 32))
    omega = np.random.default_rng(9).standard_normal((A.shape[0], 32))
    _, _, single = _single(rbl, A, 5, 32, omega, steps=6, check=False)

    def fn(ctx, r):
        ctx.set_matrix(A)
        n, r0, r1, _ = ctx.matrix_info()
        assert ctx.spmm_kernel_for(32) == 7
        Y = ctx.apply(X[r0:r1])
        _, _, info = rbl.lanczos(ctx, 5, 32, omega=omega[r0:r1], check=False, max_steps=6,
                                 trace=True, ritz=False)
        return Y, info

    parts = run_ranks(rbl, P, fn)
    Y = np.vstack([y for y, _ in parts])
    ref = A @ X
    assert np.abs(Y - ref).max() <= 1e-12 * np.abs(ref).max()
    for _, info in parts:
        for a, a1 in zip(info.trace_A + info.trace_B, single.trace_A + single.trace_B):
            assert np.abs(a - a1).max() <= 1e-10 * np.abs(a1).max()


@pytest.mark.parametrize("P,b", [(2, 8), (3, 16), (4, 32)])
def test_multirank_lanczos_matches_single_rank(rbl, P, b):
    """Full RBL run (convergence checks on, Ritz vectors) on P ranks == 1 rank == oracle."""
    k = 10
    A = matgen.hashwindow_csr(6000, 48, 0.5, 11, matgen.planted_spectrum(k))
    omega = np.random.default_rng(7).standard_normal((A.shape[0], b))
    D1, V1, info1 = _single(rbl, A, k, b, omega)
    assert info1.converged

    def fn(ctx, r):
        ctx.set_matrix(A)
        n, r0, r1, _ = ctx.matrix_info()
        D, V, info = rbl.lanczos(ctx, k, b, omega=omega[r0:r1], check=True, trace=True)
        return r0, r1, D, V, info

    parts = run_ranks(rbl, P, fn)
    for r0, r1, D, V, info in parts:
        assert info.converged and info.iters == info1.iters
        assert np.max(np.abs(D - D1) / np.abs(D1)) < 1e-10
        for a, a1 in zip(info.trace_A, info1.trace_A):
            assert np.abs(a - a1).max() <= 1e-9 * np.abs(a1).max()
    V = np.vstack([p[3] for p in parts])
    dots = np.abs(np.sum(V * V1, axis=0))
    assert np.all(1 - dots < 1e-8), dots
    ref = o.RBL_gpu_semantics(A, k, b, omega=omega, qr_mode="posdiag")
    assert np.max(np.abs(parts[0][2] - ref.D) / np.abs(ref.D)) < 1e-10


@pytest.mark.parametrize("P", [2, 4])
def test_multirank_device_generator_and_fixed_steps(rbl, P):
    """Each rank generates only its rows on the device; the fixed-step run (bench mode, block
    CGS partial reorth through the distributed Gram) matches the single-rank run."""
    n, W, p, seed, k, b = 8000, 64, 0.7734, 99, 10, 32
    plant = matgen.planted_spectrum(k)

    def fn(ctx, r):
        ctx.gen_hashwindow(n, W, p, seed, plant)
        _, _, info = rbl.lanczos(ctx, k, b, seed=5, check=False, max_steps=12, trace=True,
                                 ritz=False)
        return info

    with rbl.Context(0) as ctx:
        ctx.gen_hashwindow(n, W, p, seed, plant)
        _, _, info1 = rbl.lanczos(ctx, k, b, seed=5, check=False, max_steps=12, trace=True,
                                  ritz=False)
    infos = run_ranks(rbl, P, fn)
    for info in infos:
        assert len(info.trace_A) == len(info1.trace_A) == 12
        for a, a1 in zip(info.trace_A, info1.trace_A):
            assert np.abs(a - a1).max() <= 1e-9 * np.abs(a1).max()
        for bb, bb1 in zip(info.trace_B, info1.trace_B):
            assert np.abs(bb - bb1).max() <= 1e-9 * np.abs(bb1).max()


@pytest.mark.parametrize("bits,b", [(64, 32), (64, 16), (32, 32)])
def test_multirank_split_halo_bit_identical(rbl, bits, b):
    """RBL_OPT_SPLIT_HALO: the band-tile SpMM reading the own rows straight from the block (the
    halo buffer holds only the neighbours' rows) gives bit for bit the run that copies the own
    block into the halo buffer every step — fp64 basis and the fp32-basis direct path."""
    n, W, p, seed, k = 9000, 64, 0.7734, 41, 10
    plant = matgen.planted_spectrum(k)

    def run(split):
        def fn(ctx, r):
            ctx.set_option(rbl._lib.RBL_OPT_SPLIT_HALO, split)
            ctx.gen_hashwindow(n, W, p, seed, plant)
            assert ctx.spmm_kernel_for(b) == 5
            _, _, info = rbl.lanczos(ctx, k, b, seed=3, check=False, max_steps=10, trace=True,
                                     ritz=False, basis_bits=bits)
            return info
        return run_ranks(rbl, 3, fn)

    on, off = run(1), run(0)
    for i_on, i_off in zip(on, off):
        assert len(i_on.trace_A) == 10
        for a, a1 in zip(i_on.trace_A + i_on.trace_B, i_off.trace_A + i_off.trace_B):
            assert np.array_equal(a, a1)


@pytest.mark.parametrize("P,n,W", [(3, 150001, 64), (2, 20000, 32), (4, 700, 64)])
def test_multirank_local_reorth_fused_into_spmm(rbl, P, n, W):
    """RBL_OPT_FUSE bit 2 on several ranks: each rank corrects its first and last H rows (the
    neighbours' halo) before the exchange, the SpMM the rest as it stages them — per-step
    A_i / B_{i+1} within 1e-12 of the separate local-reorth pass (fuse 3), on ranges with and
    without an interior, H = 32 and 64, and slices shorter than 2H."""
    k, b = 10, 32
    plant = matgen.planted_spectrum(k)

    def run(fuse):
        def fn(ctx, r):
            ctx.set_option(rbl._lib.RBL_OPT_FUSE, fuse)
            ctx.gen_hashwindow(n, W, 0.7734, 17, plant)
            assert ctx.spmm_kernel_for(b) == 5
            _, _, info = rbl.lanczos(ctx, k, b, seed=9, check=False, max_steps=10, trace=True,
                                     ritz=False)
            return info
        return run_ranks(rbl, P, fn)

    fz, sep = run(7), run(3)
    for i7, i3 in zip(fz, sep):
        assert len(i7.trace_A) == len(i3.trace_A) == 10
        for t7, t3 in ((i7.trace_A, i3.trace_A), (i7.trace_B, i3.trace_B)):
            d = max(np.abs(a - a1).max() / np.abs(a1).max() for a, a1 in zip(t7, t3))
            assert d < 1e-12, d


@pytest.mark.parametrize("P", [1, 2])
def test_multirank_fused_local_reorth_runs(rbl, P):
    """The fused path really replaces the separate pass on 1 and 2 ranks (the one-wave band-tile
    SpMM; the two-waves-per-SIMD form is a variants-build kernel: test_gpu_variants).  Asserted on
    the library's path counters (rbl_path_stats), not on stage times: with both ranks on one GPU
    a stage's events also span the other rank's kernels (round 4's RBL_BT2=1 run measured rank
    0's loc-reorth stage at 2.65 ms fused against 1.46 ms separate — about one of rank 1's SpMM
    launches per step, ~0.37 ms at 1e6 rows, waiting in front of rank 0's small fix-up kernels
    while the persistent SpMM held every CU's LDS).  Fused (RBL_OPT_FUSE 7): every step from
    i = 2 on applies the update inside the SpMM, fixes the range edges after it (and on several
    ranks the rank edges before the exchange), and runs no separate pass; unfused (3): a
    separate pass per step and no fused SpMM.  Both give the same A_i / B_{i+1} to 1e-12."""
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
        assert p7["spmm_two_wave"] == p3["spmm_two_wave"] == 0
        for a, a1 in zip(i7.trace_A + i7.trace_B, i3.trace_A + i3.trace_B):
            assert np.abs(a - a1).max() <= 1e-12 * np.abs(a1).max()


def test_multirank_tiny_slices(rbl):
    """More ranks than comfortable: 4 ranks on n = 12 (3 rows each), b = 4."""
    import scipy.sparse as sp
    rng = np.random.default_rng(3)
    M = rng.standard_normal((12, 12))
    A = sp.csr_matrix(M + M.T)
    omega = rng.standard_normal((12, 4))
    D1, V1, info1 = _single(rbl, A, 2, 4, omega, check=False, steps=2)

    def fn(ctx, r):
        ctx.set_matrix(A)
        _, r0, r1, _ = ctx.matrix_info()
        _, _, info = rbl.lanczos(ctx, 2, 4, omega=omega[r0:r1], check=False, max_steps=2,
                                 trace=True, ritz=False)
        return info

    for info in run_ranks(rbl, 4, fn):
        for a, a1 in zip(info.trace_A, info1.trace_A):
            assert np.abs(a - a1).max() <= 1e-10 * np.abs(a1).max()


def test_rccl_transport_selftest(rbl):
    """The production transport (RcclComm over RCCL): ncclCommInitRank at one rank, then the
    three collective shapes of a row-partitioned step — in-place all-reduce of fp64 device
    data, host all-gather of int64, an (empty) grouped send/recv — checked on the host."""
    import ctypes
    from rbl import _lib
    msg = ctypes.create_string_buffer(256)
    st = _lib.lib.rbl_comm_selftest(0, msg, 256)
    assert st == _lib.RBL_OK, msg.value.decode()
    assert msg.value.decode() == "ok: rccl"


def test_multirank_matrix_sequence_like_bench(rbl):
    """bench.py's sequence on one context per rank: the hash-window run, then the R-MAT and the
    circuit sub-records, each matrix generated in place of the last (every plan — halo, tiers,
    basis — rebuilt).  On 2 in-process ranks each fixed-step trace equals the single-rank one."""
    from oracle import matgen
    plant = matgen.planted_spectrum(5)
    gens = [lambda c: c.gen_hashwindow(3000, 64, 0.7734, 5, plant),
            lambda c: c.gen_rmat(6000, 13, 120_000, 7, plant),
            lambda c: c.gen_circuit(5000, 5, plant, width=71)]
    shapes = [(32, 6), (32, 6), (16, 6)]

    def run(ctx):
        out = []
        for g, (b, steps) in zip(gens, shapes):
            g(ctx)
            _, _, info = rbl.lanczos(ctx, 5, b, seed=3, check=False, max_steps=steps, trace=True,
                                     ritz=False)
            out.append(info)
        return out

    with rbl.Context(0) as ctx:
        single = run(ctx)
    for per_rank in run_ranks(rbl, 2, lambda ctx, r: run(ctx)):
        for info, ref in zip(per_rank, single):
            for a, a1 in zip(info.trace_A, ref.trace_A):
                assert np.abs(a - a1).max() <= 1e-9 * np.abs(a1).max()
            for bb, bb1 in zip(info.trace_B, ref.trace_B):
                assert np.abs(bb - bb1).max() <= 1e-9 * np.abs(bb1).max()


def test_start_allocation_failure_is_collective(rbl):
    """A run whose buffers do not fit on one rank: rbl_start votes on its allocations before the
    collectives of the start, so every rank returns RBL_ERR_OOM (the peers naming the rank that
    failed) instead of waiting in the halo exchange for it; the contexts then run a normal start.
    (Rank 0 keeps every block in HBM, RBL_OPT_DEVICE_BLOCKS = 0, for 321 blocks of 1 GB; rank 1
    keeps 3 and would spill the rest, which fits.)"""
    from rbl import _lib
    plant = np.array([100.0 * (7 - l) for l in range(1, 7)])

    def fn(ctx, r):
        ctx.gen_hashwindow(8_000_000, 16, 0.5, 3, plant)
        ctx.set_option(_lib.RBL_OPT_DEVICE_BLOCKS, 0 if r == 0 else 3)
        err = None
        try:
            ctx.start(32, 320)
        except rbl.RBLError as e:
            err = (e.code, str(e))
        ctx.set_option(_lib.RBL_OPT_DEVICE_BLOCKS, 0)
        _, _, info = rbl.lanczos(ctx, 3, 32, seed=1, check=False, max_steps=3, trace=True,
                                 ritz=False)
        return err, info

    out = run_ranks(rbl, 2, fn)
    assert out[0][0] is not None and out[0][0][0] == _lib.RBL_ERR_OOM
    assert out[1][0] is not None and out[1][0][0] == _lib.RBL_ERR_OOM and "rank 0" in out[1][0][1]
    for a, a1 in zip(out[0][1].trace_A, out[1][1].trace_A):
        assert np.array_equal(a, a1)
