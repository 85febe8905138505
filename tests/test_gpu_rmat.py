"""GPU: the R-MAT generator (BASELINE config 4) and the Lanczos path on a
power-law pattern.

The device generator must match the NumPy restatement (oracle/matgen.py rmat_csr) bit for bit
(integer structure and fp64 values), on one rank and on nnz-balanced row slices of several
in-process ranks.  SpMM: every element within 1e-13 (|A| |X|) of SciPy.  Eigenvalues: 1e-10
relative against the oracle (parity unpinned beyond the restatement: the reference has no
R-MAT fixture)."""
import os

import numpy as np
import pytest

from oracle import matgen
from oracle import rbl_oracle as o
from test_gpu_multirank import run_ranks

pytestmark = pytest.mark.gpu

CASE = dict(n=6000, scale=13, edges=120_000, seed=7)


@pytest.fixture(scope="module")
def rbl():
    import rbl as _r
    return _r


def _csr_equal(ref, rowptr, col, val):
    assert np.array_equal(ref.indptr, rowptr)
    assert np.array_equal(ref.indices, col)
    assert np.array_equal(ref.data, val)


def test_rmat_generator_bit_exact(rbl):
    plant = matgen.planted_spectrum(5)
    ref = matgen.rmat_csr(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
    with rbl.Context(0) as ctx:
        ctx.gen_rmat(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
        n, r0, r1, nnz = ctx.matrix_info()
        assert (n, r0, r1, nnz) == (CASE["n"], 0, CASE["n"], ref.nnz)
        _csr_equal(ref, *ctx.get_matrix_csr())
        assert ctx.spmm_kernel_for(32) == 6   # unbanded: the segmented gather


@pytest.mark.parametrize("P", [2, 3])
def test_rmat_generator_ranks_balanced(rbl, P):
    """Each rank generates its own rows; slices tile [0, n) and split the nonzeros about evenly
    (balanced on the draw counts before duplicates merge: within 25 % of the mean, and better
    than a uniform row split, which puts the hubs' rows on rank 0)."""
    plant = matgen.planted_spectrum(5)
    full = matgen.rmat_csr(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)

    def fn(ctx, r):
        ctx.gen_rmat(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
        _, r0, r1, nnz = ctx.matrix_info()
        return r0, r1, nnz, ctx.get_matrix_csr()

    parts = run_ranks(rbl, P, fn)
    assert parts[0][0] == 0 and parts[-1][1] == CASE["n"]
    for (r0, r1, nnz, csr), nxt in zip(parts, parts[1:] + [None]):
        if nxt is not None:
            assert r1 == nxt[0]
        _csr_equal(full[r0:r1], *csr)
        assert abs(nnz - full.nnz / P) < 0.25 * full.nnz / P
    uniform = max(full[CASE["n"] * q // P: CASE["n"] * (q + 1) // P].nnz for q in range(P))
    assert max(p[2] for p in parts) < uniform


@pytest.mark.parametrize("b", [8, 16, 32])
def test_rmat_spmm(rbl, b):
    A = matgen.rmat_csr(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"])
    X = np.random.default_rng(b).standard_normal((A.shape[0], b))
    with rbl.Context(0) as ctx:
        ctx.gen_rmat(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"])
        Y = ctx.apply(X)
    ref = A @ X
    bound = (abs(A) @ np.abs(X)) * 1e-13 + 1e-300
    assert np.all(np.abs(Y - ref) <= bound)


def test_rmat_lanczos_matches_oracle(rbl):
    k, b = 10, 16
    plant = matgen.planted_spectrum(k)
    A = matgen.rmat_csr(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
    omega = np.random.default_rng(3).standard_normal((A.shape[0], b))
    with rbl.Context(0) as ctx:
        ctx.gen_rmat(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
        D, V, info = rbl.lanczos(ctx, k, b, omega=omega, check=True)
    ref = o.RBL_gpu_semantics(A, k, b, omega=omega, qr_mode="posdiag", reorth_mode="cgs")
    assert info.converged and ref.converged
    assert np.max(np.abs(D - ref.D) / np.abs(ref.D)) < 1e-10
    res = np.linalg.norm(A @ V - V * D, axis=0) / np.abs(D)
    assert res.max() < 1e-7


def test_rmat_multirank_lanczos(rbl):
    """C4b's multi-GPU form (BASELINE config 4): each rank generates its nnz-balanced rows, the
    halo exchange brings in every Q row its columns touch (for R-MAT nearly all of them), the
    segmented gather multiplies; the fixed-step trace equals the single-rank run's."""
    plant = matgen.planted_spectrum(5)

    def run(ctx):
        ctx.gen_rmat(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
        _, _, info = rbl.lanczos(ctx, 5, 32, seed=9, check=False, max_steps=8, trace=True,
                                 ritz=False)
        return info

    with rbl.Context(0) as ctx:
        info1 = run(ctx)
    for info in run_ranks(rbl, 3, lambda ctx, r: run(ctx)):
        for a, a1 in zip(info.trace_A, info1.trace_A):
            assert np.abs(a - a1).max() <= 1e-9 * np.abs(a1).max()
        for bb, bb1 in zip(info.trace_B, info1.trace_B):
            assert np.abs(bb - bb1).max() <= 1e-9 * np.abs(bb1).max()


@pytest.mark.parametrize("P", [2, 3])
def test_rmat_multirank_halo_overlap_bit_identical(rbl, P):
    """Several ranks on an unbanded matrix: each rank's SpMM runs as two column tiers, the own
    columns (gathered from the block itself while the halo exchange is in flight on a side
    stream) and the halo columns (after the exchange lands), renumbered to the ghost rows the
    indexed halo delivers — only the rows a rank's columns reference.  RBL_OPT_HALO_OVERLAP only moves
    the exchange off the SpMM's stream, so A_i / B_i are bit-identical with it on and off, and
    equal the single-rank run to rounding; the collective counters see one exchange per SpMM."""
    from rbl import _lib
    plant = matgen.planted_spectrum(5)
    steps = 8

    def run(overlap):
        def fn(ctx, r):
            ctx.set_option(_lib.RBL_OPT_HALO_OVERLAP, overlap)
            ctx.set_option(_lib.RBL_OPT_HALO_PUSH, 0)   # the pull-all halo (counted below)
            ctx.gen_rmat(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
            _, r0, r1, _ = ctx.matrix_info()
            _, col, _ = ctx.get_matrix_csr()
            ghosts = np.unique(col[(col < r0) | (col >= r1)]).size
            ctx.comm_stats(reset=True)
            _, _, info = rbl.lanczos(ctx, 5, 32, seed=9, check=False, max_steps=steps,
                                     trace=True, ritz=False)
            return info, ctx.comm_stats(), ghosts
        return run_ranks(rbl, P, fn)

    on, off = run(1), run(0)
    with rbl.Context(0) as ctx:
        ctx.gen_rmat(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
        _, _, single = rbl.lanczos(ctx, 5, 32, seed=9, check=False, max_steps=steps, trace=True,
                                   ritz=False)
    for (i_on, st_on, ghosts), (i_off, st_off, _) in zip(on, off):
        for a, a0 in zip(i_on.trace_A + i_on.trace_B, i_off.trace_A + i_off.trace_B):
            assert np.array_equal(a, a0)
        for a, a1 in zip(i_on.trace_A, single.trace_A):
            assert np.abs(a - a1).max() <= 1e-9 * np.abs(a1).max()
        assert st_on == st_off
        assert st_on["exchange_calls"] == steps + 1      # rbl_start + one per block step
        # indexed halo: each exchange receives exactly the rows the rank's columns reference
        assert st_on["recv_bytes"] == (steps + 1) * ghosts * 32 * 8 > 0
        assert st_on["allreduce_calls"] >= 4 * (steps - 1)


def test_rmat_indexed_halo_small_and_ragged(rbl):
    """The indexed halo at the edges: n = 700 on 4 ranks (a hub-heavy first rank with few
    rows, peers that need nothing from some ranks), b = 16 and b = 32; the fixed-step traces
    equal the single-rank ones, and rbl_apply through the ghost exchange matches SciPy."""
    plant = matgen.planted_spectrum(3)
    n, scale, edges, seed = 700, 10, 30_000, 13
    A = matgen.rmat_csr(n, scale, edges, seed, plant)
    X = np.random.default_rng(5).standard_normal((n, 16))
    for b in (16, 32):
        def run(ctx):
            ctx.gen_rmat(n, scale, edges, seed, plant)
            _, _, info = rbl.lanczos(ctx, 3, b, seed=2, check=False, max_steps=6, trace=True,
                                     ritz=False)
            return info

        with rbl.Context(0) as ctx:
            ref = run(ctx)

        def fn(ctx, r):
            info = run(ctx)
            _, r0, r1, _ = ctx.matrix_info()
            return info, r0, r1

        out = run_ranks(rbl, 4, fn)
        for info, _, _ in out:
            for a, a1 in zip(info.trace_A, ref.trace_A):
                assert np.abs(a - a1).max() <= 1e-9 * np.abs(a1).max()

    def fa(ctx, r):
        ctx.gen_rmat(n, scale, edges, seed, plant)
        _, r0, r1, _ = ctx.matrix_info()
        return r0, ctx.apply(X[r0:r1])

    parts = sorted(run_ranks(rbl, 4, fa), key=lambda t: t[0])
    Y = np.vstack([y for _, y in parts])
    bound = (abs(A) @ np.abs(X)) * 1e-13 + 1e-300
    assert np.all(np.abs(Y - A @ X) <= bound)


def test_rmat_relabel_generator_bit_exact(rbl):
    """RBL_OPT_RELABEL = 1: the device generator stores P A P^T (vertex v at row / column
    perm(v)), bit for bit the restatement matgen.rmat_csr(relabel=True), on one rank and on the
    nnz-balanced slices of 3 ranks; rbl_row_ids returns perm^-1 of the local rows."""
    from rbl import _lib
    plant = matgen.planted_spectrum(5)
    ref = matgen.rmat_csr(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant,
                          relabel=True)
    perm_inv = matgen.rmat_relabel(CASE["n"], CASE["seed"], np.arange(CASE["n"]), inverse=True)

    def fn(ctx, r):
        ctx.set_option(_lib.RBL_OPT_RELABEL, 1)
        ctx.gen_rmat(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
        _, r0, r1, _ = ctx.matrix_info()
        return r0, r1, ctx.get_matrix_csr(), ctx.row_ids()

    with rbl.Context(0) as ctx:
        r0, r1, csr, ids = fn(ctx, 0)
    assert (r0, r1) == (0, CASE["n"])
    _csr_equal(ref, *csr)
    assert np.array_equal(ids, perm_inv)
    for r0, r1, csr, ids in run_ranks(rbl, 3, fn):
        _csr_equal(ref[r0:r1], *csr)
        assert np.array_equal(ids, perm_inv[r0:r1])


def test_rmat_relabel_is_the_plain_run_permuted(rbl):
    """The relabelled matrix with the device start block (drawn per original id) runs the plain
    run's Krylov sequence with its rows permuted: per-step A_i / B_{i+1} to 1e-9 (the SpMM sums
    a row's nonzeros in another column order), eigenvalues < 1e-10, and the Ritz vectors, put
    back in original row order by rbl_row_ids, equal up to sign (1 - |v.v'| < 1e-8)."""
    from rbl import _lib
    k, b = 10, 32
    plant = matgen.planted_spectrum(k)
    n, scale, edges, seed = 60000, 16, 60000 * 66, 7
    out = {}
    for rl in (0, 1):
        with rbl.Context(0) as ctx:
            ctx.set_option(_lib.RBL_OPT_RELABEL, rl)
            ctx.gen_rmat(n, scale, edges, seed, plant)
            ids = ctx.row_ids()
            D, V, info = rbl.lanczos(ctx, k, b, seed=4, check=True, trace=True)
            Vo = np.zeros_like(V)
            Vo[ids] = V
            out[rl] = (D, Vo, info)
    (D0, V0, i0), (D1, V1, i1) = out[0], out[1]
    assert i0.converged and i1.converged and i0.iters == i1.iters
    assert np.max(np.abs(D1 - D0) / np.abs(D0)) < 1e-10
    for a, a0 in zip(i1.trace_A + i1.trace_B, i0.trace_A + i0.trace_B):
        assert np.abs(a - a0).max() <= 1e-9 * np.abs(a0).max()
    assert np.all(1 - np.abs(np.sum(V0 * V1, axis=0)) < 1e-8)


def test_rmat_relabel_balances_the_halo(rbl):
    """The reason for the relabel (BASELINE config 4 on 8 GPUs): with R-MAT's hubs at the low ids
    the nnz-balanced split gives one rank most of the rows its peers reference, so it sends far
    more than the others.  Relabelled, the busiest sender is within 1.2x the mean on 4 and 8
    in-process ranks (n = 2e5, the bench's draw density), and the traces match the single-rank
    relabelled run."""
    from rbl import _lib
    n, scale, edges, seed = 200_000, 18, int(0.66 * 100 * 200_000), 20261015
    plant = matgen.planted_spectrum(5)
    for P in (4, 8):
        sends = {}
        for rl in (0, 1):
            def fn(ctx, r):
                ctx.set_option(_lib.RBL_OPT_RELABEL, rl)
                ctx.set_option(_lib.RBL_OPT_HALO_PUSH, 0)   # the pull-all halo's balance
                ctx.gen_rmat(n, scale, edges, seed, plant)
                ctx.comm_stats(reset=True)
                _, _, info = rbl.lanczos(ctx, 5, 32, seed=9, check=False, max_steps=4, trace=True,
                                         ritz=False)
                return ctx.comm_stats()["send_bytes"], info
            res = run_ranks(rbl, P, fn, timeout=400)
            sends[rl] = np.array([s for s, _ in res], dtype=float)
        ratio0 = sends[0].max() / sends[0].mean()
        ratio1 = sends[1].max() / sends[1].mean()
        print(f"P={P}: busiest sender / mean: plain {ratio0:.2f}, relabelled {ratio1:.2f}")
        assert ratio1 <= 1.2 < ratio0


@pytest.mark.parametrize("b,kernel", [(8, 0), (32, 1), (16, 1), (40, 0)])
def test_rmat_multirank_range_halo_beside_ghosts(rbl, b, kernel):
    """A ghost-built (indexed-halo) context still runs every block size and kernel: for b outside
    {16, 32}, or the gather pinned by RBL_OPT_SPMM_KERNEL = 1, the ranks use the range halo kept
    beside the ghost tables (all ranks pick the same exchange); traces equal the single-rank
    run's, and rbl_apply matches SciPy."""
    from rbl import _lib
    plant = matgen.planted_spectrum(3)
    A = matgen.rmat_csr(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
    X = np.random.default_rng(b).standard_normal((CASE["n"], b))

    def run(ctx):
        ctx.set_option(_lib.RBL_OPT_SPMM_KERNEL, kernel)
        ctx.gen_rmat(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
        assert ctx.spmm_kernel_for(b) == 1
        _, _, info = rbl.lanczos(ctx, 3, b, seed=2, check=False, max_steps=6, trace=True,
                                 ritz=False)
        return info

    with rbl.Context(0) as ctx:
        ref = run(ctx)

    def fn(ctx, r):
        info = run(ctx)
        _, r0, r1, _ = ctx.matrix_info()
        return info, r0, ctx.apply(X[r0:r1])

    out = run_ranks(rbl, 3, fn)
    for info, _, _ in out:
        for a, a1 in zip(info.trace_A, ref.trace_A):
            assert np.abs(a - a1).max() <= 1e-9 * np.abs(a1).max()
    Y = np.vstack([y for _, _, y in sorted(out, key=lambda t: t[1])])
    bound = (abs(A) @ np.abs(X)) * 1e-13 + 1e-300
    assert np.all(np.abs(Y - A @ X) <= bound)


def _scattered(n, live, seed=6):
    """A symmetric scattered pattern on the first `live` rows (~30 nonzeros per row, no band,
    no window fit: every SpMM format votes unbanded) and empty rows after them."""
    import scipy.sparse as sp
    rng = np.random.default_rng(seed)
    R = sp.random(live, live, density=15 / live, random_state=seed, format="csr")
    R = R + R.T + sp.diags(rng.uniform(1, 2, live))
    M = sp.block_diag([R, sp.csr_matrix((n - live, n - live))]).tocsr()
    M.sort_indices()
    return M


def test_unbanded_ranks_without_rows_or_nonzeros(rbl):
    """The setup collectives when some ranks hold nothing: an unbanded (scattered) user CSR on 4
    ranks whose caller-given row split leaves two ranks with rows but no nonzeros, and a matrix
    with n < P that leaves a rank without rows.  Every rank takes part in the banded vote and
    the ghost exchange (the pull-all indexed halo here); the traces equal the single-rank run's."""
    import scipy.sparse as sp
    from rbl import _lib
    rng = np.random.default_rng(5)
    n, live = 4000, 3000
    M = _scattered(n, live)
    omega = rng.standard_normal((n, 16))
    with rbl.Context(0) as ctx:
        ctx.set_matrix(M)
        _, _, ref = rbl.lanczos(ctx, 3, 16, omega=omega, check=False, max_steps=5, trace=True,
                                ritz=False)
    bounds = [0, 1500, 3000, 3500, 4000]

    def fn(ctx, r):
        r0, r1 = bounds[r], bounds[r + 1]
        S = M[r0:r1]
        ctx.set_option(_lib.RBL_OPT_HALO_PUSH, 0)
        ctx.set_matrix_rows(n, r0, r1, S.indptr, S.indices, S.data)
        _, _, _, nnz = ctx.matrix_info()
        ctx.comm_stats(reset=True)
        _, _, info = rbl.lanczos(ctx, 3, 16, omega=omega[r0:r1], check=False, max_steps=5,
                                 trace=True, ritz=False)
        return info, nnz, ctx.spmm_kernel_for(16), ctx.comm_stats()

    out = run_ranks(rbl, 4, fn)
    assert [nnz == 0 for _, nnz, _, _ in out] == [False, False, True, True]
    assert out[0][2] == 6       # the segmented gather with the indexed halo on the live ranks
    # the unbanded vote held on every rank: the indexed halo moves the referenced rows only
    assert out[0][3]["pull_rows_pred"] > 0
    assert sum(st["recv_bytes"] for *_, st in out) == 6 * out[0][3]["pull_rows_pred"] * 16 * 8
    for info, _, _, _ in out:
        for a, a1 in zip(info.trace_A, ref.trace_A):
            assert np.abs(a - a1).max() <= 1e-9 * np.abs(a1).max()

    # n < P: a rank with no rows at all
    T = sp.csr_matrix(np.array([[2.0, 1, 0], [1, 3, 0], [0, 0, 4]]))
    om = rng.standard_normal((3, 2))
    with rbl.Context(0) as ctx:
        ctx.set_matrix(T)
        _, _, ref = rbl.lanczos(ctx, 1, 2, omega=om, check=False, max_steps=1, trace=True,
                                ritz=False)

    def fn2(ctx, r):
        ctx.set_matrix(T)
        _, r0, r1, _ = ctx.matrix_info()
        _, _, info = rbl.lanczos(ctx, 1, 2, omega=om[r0:r1], check=False, max_steps=1,
                                 trace=True, ritz=False)
        return info, r1 - r0

    out = run_ranks(rbl, 4, fn2)
    assert any(m == 0 for _, m in out)
    for info, _ in out:
        assert np.abs(info.trace_A[0] - ref.trace_A[0]).max() <= 1e-12 * np.abs(ref.trace_A[0]).max()


def _push_plan(A, bounds):
    """The push/pull split's moved rows per SpMM (summed over ranks) restated from the full CSR:
    rank p pulls the off-rank columns c of its rows r with (deg c, -c) > (deg r, -r) and pushes
    as many partial rows; the pull-all halo moves every distinct off-rank column."""
    deg = np.diff(A.indptr)
    push = pull = 0
    for r0, r1 in zip(bounds[:-1], bounds[1:]):
        S = A[r0:r1].tocoo()
        rows, cols = S.row + r0, S.col
        off = (cols < r0) | (cols >= r1)
        rows, cols = rows[off], cols[off]
        up = (deg[cols] > deg[rows]) | ((deg[cols] == deg[rows]) & (cols < rows))
        push += 2 * np.unique(cols[up]).size
        pull += np.unique(cols).size
    return push, pull


@pytest.mark.parametrize("P", [2, 3, 4])
def test_rmat_halo_push_split(rbl, P):
    """RBL_OPT_HALO_PUSH: the hub-aware push/pull split of the indexed halo.  Each off-rank
    product is formed on the rank of its higher-(degree, id) endpoint — pulled Q rows for the
    columns above the row, pushed partial rows (the push tier: the pulled entries transposed)
    for the rest.  Checked: the moved rows per SpMM equal the restated plan and the exchanges'
    byte counts (send = recv on every rank: the push mirrors the pull), two exchanges per SpMM,
    A_i / B_{i+1} bit-identical with the side stream on and off, equal to the pull-all halo and
    the single-rank run to 1e-9 (only the order of each row's sum differs), and rbl_apply
    through the split within 1e-13 |A||X| of SciPy."""
    from rbl import _lib
    plant = matgen.planted_spectrum(5)
    A = matgen.rmat_csr(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
    X = np.random.default_rng(3).standard_normal((CASE["n"], 32))
    steps, b = 8, 32

    def run(push, overlap):
        def fn(ctx, r):
            ctx.set_option(_lib.RBL_OPT_HALO_OVERLAP, overlap)
            ctx.set_option(_lib.RBL_OPT_HALO_PUSH, push)
            ctx.gen_rmat(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
            _, r0, r1, _ = ctx.matrix_info()
            Y = ctx.apply(X[r0:r1])
            ctx.comm_stats(reset=True)
            _, _, info = rbl.lanczos(ctx, 5, b, seed=9, check=False, max_steps=steps,
                                     trace=True, ritz=False)
            return info, ctx.comm_stats(), r0, r1, Y
        return run_ranks(rbl, P, fn)

    on, seq, pull = run(1, 1), run(1, 0), run(0, 1)
    with rbl.Context(0) as ctx:
        ctx.gen_rmat(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
        _, _, single = rbl.lanczos(ctx, 5, b, seed=9, check=False, max_steps=steps, trace=True,
                                   ritz=False)
    bounds = [r0 for _, _, r0, _, _ in on] + [CASE["n"]]
    want_push, want_pull = _push_plan(A, bounds)
    print(f"P={P}: rows moved per SpMM: push/pull split {want_push}, pull-all {want_pull}")
    for (i_on, st, _, _, _), (i_seq, st_seq, _, _, _), (i_pl, st_pl, _, _, _) in zip(on, seq, pull):
        for a, a0 in zip(i_on.trace_A + i_on.trace_B, i_seq.trace_A + i_seq.trace_B):
            assert np.array_equal(a, a0)
        for a, a1, a2 in zip(i_on.trace_A, single.trace_A, i_pl.trace_A):
            assert np.abs(a - a1).max() <= 1e-9 * np.abs(a1).max()
            assert np.abs(a - a2).max() <= 1e-9 * np.abs(a2).max()
        assert st["halo_push"] == 1 and st_pl["halo_push"] == 0
        assert (st["push_rows_pred"], st["pull_rows_pred"]) == (want_push, want_pull)
        assert st["exchange_calls"] == 2 * (steps + 1) and st_pl["exchange_calls"] == steps + 1
        assert st["send_bytes"] == st["recv_bytes"] and st == st_seq
    moved = sum(st["recv_bytes"] for _, st, _, _, _ in on) // ((steps + 1) * b * 8)
    moved_pl = sum(st["recv_bytes"] for _, st, _, _, _ in pull) // ((steps + 1) * b * 8)
    assert (moved, moved_pl) == (want_push, want_pull)
    bound = (abs(A) @ np.abs(X)) * 1e-13 + 1e-300
    for res in (on, seq):
        Y = np.vstack([y for _, _, _, _, y in res])
        assert np.all(np.abs(Y - A @ X) <= bound)


def test_rmat_halo_push_small_and_ragged(rbl):
    """The split at the edges: n = 700 on 4 ranks with b = 16 and 32 (peers that push nothing to
    some ranks), and a user CSR whose caller-given split leaves ranks with rows but no nonzeros
    and one with no rows at all (n = 3, P = 4); the traces equal the single-rank ones."""
    import scipy.sparse as sp
    from rbl import _lib
    plant = matgen.planted_spectrum(3)
    n, scale, edges, seed = 700, 10, 30_000, 13
    for b in (16, 32):
        def run(ctx):
            ctx.set_option(_lib.RBL_OPT_HALO_PUSH, 1)
            ctx.gen_rmat(n, scale, edges, seed, plant)
            _, _, info = rbl.lanczos(ctx, 3, b, seed=2, check=False, max_steps=6, trace=True,
                                     ritz=False)
            return info, ctx.comm_stats()["halo_push"]

        with rbl.Context(0) as ctx:
            ref, _ = run(ctx)
        for info, hp in run_ranks(rbl, 4, lambda ctx, r: run(ctx)):
            assert hp == 1
            for a, a1 in zip(info.trace_A, ref.trace_A):
                assert np.abs(a - a1).max() <= 1e-9 * np.abs(a1).max()
    rng = np.random.default_rng(5)
    n, live = 4000, 3000
    M = _scattered(n, live)
    omega = rng.standard_normal((n, 16))
    with rbl.Context(0) as ctx:
        ctx.set_matrix(M)
        _, _, ref = rbl.lanczos(ctx, 3, 16, omega=omega, check=False, max_steps=5, trace=True,
                                ritz=False)
    for bounds in ([0, 1500, 3000, 3500, 4000], [0, 1000, 2000, 3000, 4000]):
        def fn(ctx, r):
            r0, r1 = bounds[r], bounds[r + 1]
            S = M[r0:r1]
            ctx.set_option(_lib.RBL_OPT_HALO_PUSH, 1)
            ctx.set_matrix_rows(n, r0, r1, S.indptr, S.indices, S.data)
            _, _, info = rbl.lanczos(ctx, 3, 16, omega=omega[r0:r1], check=False, max_steps=5,
                                     trace=True, ritz=False)
            return info, ctx.comm_stats()["halo_push"]
        for info, hp in run_ranks(rbl, 4, fn):
            assert hp == 1
            for a, a1 in zip(info.trace_A, ref.trace_A):
                assert np.abs(a - a1).max() <= 1e-9 * np.abs(a1).max()


@pytest.mark.parametrize("kind", ["pattern", "value", "swap"])
def test_rmat_halo_push_needs_symmetric_pattern(rbl, kind):
    """The split relies on A[c, r] = A[r, c] (the owner of c forms the product from its own row).
    A matrix that is not symmetric across ranks is caught at setup — by the per-pair entry
    counts, and by per-pair hashes of the entries themselves (row, column, value bits): one
    entry without its mirror ("pattern"), a mirrored pair with different values ("value"), two
    unmirrored entries in opposite directions ("swap": the per-pair counts may still agree).
    RBL_OPT_HALO_PUSH 1 fails with a message, the automatic mode keeps the pull-all halo (and
    the product stays exact)."""
    import scipy.sparse as sp
    from rbl import _lib
    rng = np.random.default_rng(2)
    n = 3000
    M = _scattered(n, n, seed=4)
    free = [j for j in range(1500, n) if M[5, j] == 0 and M[j, 5] == 0]
    j, j2 = free[0], free[1]
    M = M.tolil()
    if kind == "pattern":
        M[5, j] = 0.7            # one entry without its mirror, across the ranks' boundary
    elif kind == "value":
        M[5, j], M[j, 5] = 0.7, 0.7000000000000001   # mirrored, one ulp apart
    else:
        M[5, j], M[j2, 5] = 0.7, 0.7
    M = M.tocsr()
    M.sort_indices()
    X = rng.standard_normal((n, 16))
    bounds = [0, 1500, 3000]

    def fn(mode):
        def f(ctx, r):
            r0, r1 = bounds[r], bounds[r + 1]
            Sr = M[r0:r1]
            ctx.set_option(_lib.RBL_OPT_HALO_PUSH, mode)
            try:
                ctx.set_matrix_rows(n, r0, r1, Sr.indptr, Sr.indices, Sr.data)
            except Exception as e:  # noqa: BLE001 - the failure is the result
                return str(e)
            return ctx.comm_stats()["halo_push"], ctx.apply(X[r0:r1])
        return run_ranks(rbl, 2, f)

    forced = fn(1)
    assert all(isinstance(x, str) and "symmetric" in x for x in forced), forced
    auto = fn(2)
    assert all(hp == 0 for hp, _ in auto)
    Y = np.vstack([y for _, y in auto])
    bound = (abs(M) @ np.abs(X)) * 1e-13 + 1e-300
    assert np.all(np.abs(Y - M @ X) <= bound)


def test_push_buffer_allocation_failure_is_collective(rbl, monkeypatch):
    """The push/pull split's partial-row buffers are allocated inside rbl_start's allocation
    vote (not lazily in the first push exchange): when rank 1 cannot allocate them
    (RBL_FAULT_PUSH_ALLOC=1 injects the failure at exactly that allocation) every rank returns
    RBL_ERR_OOM from rbl_start — rank 0 naming rank 1 — instead of rank 0 waiting in the push
    exchange for a rank that has left; a normal run then follows on the same contexts."""
    from rbl import _lib
    plant = matgen.planted_spectrum(5)

    def fn(ctx, r):
        ctx.set_option(_lib.RBL_OPT_HALO_PUSH, 1)
        ctx.gen_rmat(CASE["n"], CASE["scale"], CASE["edges"], CASE["seed"], plant)
        err = None
        try:
            ctx.start(32, 8, seed=9)
        except rbl.RBLError as e:
            err = (e.code, str(e))
        barrier.wait(timeout=60)           # both ranks are past the failed start
        if r == 0:
            os.environ.pop("RBL_FAULT_PUSH_ALLOC", None)
        barrier.wait(timeout=60)
        _, _, info = rbl.lanczos(ctx, 5, 32, seed=9, check=False, max_steps=4, trace=True,
                                 ritz=False)
        return err, info, ctx.comm_stats()

    import threading
    barrier = threading.Barrier(2)
    monkeypatch.setenv("RBL_FAULT_PUSH_ALLOC", "1")
    out = run_ranks(rbl, 2, fn)
    assert out[1][0] is not None and out[1][0][0] == _lib.RBL_ERR_OOM and "injected" in out[1][0][1]
    assert out[0][0] is not None and out[0][0][0] == _lib.RBL_ERR_OOM and "rank 1" in out[0][0][1]
    for a, a1 in zip(out[0][1].trace_A, out[1][1].trace_A):
        assert np.array_equal(a, a1)
    assert all(st["halo_push"] == 1 for _, _, st in out)
