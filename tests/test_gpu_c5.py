"""GPU: BASELINE config 5 at its own size on ONE MI355X — n = 5e7, ~100 nnz/row (5.0e9
nonzeros: int64 row pointers, nonzero offsets past 2^32), b = 32, k = 20, the mixed-precision
path (FLOAT = Float32 basis, fp64 A*Q / 3-term / QR: RBL_gpu.jl with common.jl:5 FLOAT =
Float32).  The oracle cannot run at this size, so size-independent properties:

  * memory plan: the CSR (60 GB) is released once the band tiles are built
    (RBL_OPT_KEEP_CSR = 0) and the fp32 basis spills to pinned host memory beyond a few device
    slots (RBL_OPT_DEVICE_BLOCKS, the reference's FLOAT hybrid buffer, RBL_gpu.jl:59-81);
  * SpMM (the band-tile kernel of the run) on sampled row windows — first rows, the ragged last
    tile, and windows spread over all 5e7 rows — against SciPy on the same rows produced by the
    host twin of the device generator (bit-identical generator: test_lib_host), every element
    within 1e-13 * (|A| |X|);
  * the mixed RBL_gpu to convergence: the planted top spectrum found, residuals
    ||A v - lambda v|| / |lambda| < 1e-5 (A v by the device SpMM verified above), Ritz vectors
    orthonormal within 1e-5, Rayleigh quotients within 1e-5 relative, D descending by |lambda|.

Device memory ~120 GB (band tiles 57.5 GB + fp64 working blocks + a few fp32 slots); host
~45 GB (X, A X, V, the spilled slots)."""
import time

import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu

N, HALFWIDTH, DENSITY, SEED, B, K = 50_000_000, 64, 0.7734, 20261015, 32, 20
DEVICE_BLOCKS = 6           # 4 resident fp32 blocks + 2 working slots; older blocks spill
SPMM_TOL = 1e-13
# the Ritz vectors are combinations of fp32-rounded blocks: v^T v - 1 and v^T A v / v^T v -
# lambda sit at the basis' orthogonality level (~1e-6 measured), so both are held to 1e-5
RES_TOL, ORTH_TOL, RAYLEIGH_TOL = 1e-5, 1e-5, 1e-5
T0 = time.perf_counter()
PLANT = np.array([100.0 * (2 * K + 1 - l) for l in range(1, 2 * K + 1)])


def log(msg):
    print(f"[c5] {msg} {time.perf_counter() - T0:.1f} s", flush=True)


@pytest.fixture(scope="module")
def c5():
    import rbl
    ctx = rbl.Context(0)
    ctx.set_option(rbl._lib.RBL_OPT_KEEP_CSR, 0)
    ctx.gen_hashwindow(N, HALFWIDTH, DENSITY, SEED, PLANT)
    n, r0, r1, nnz = ctx.matrix_info()
    assert (n, r0, r1) == (N, 0, N) and 4.95e9 < nnz < 5.05e9
    log(f"generated {nnz} nonzeros")
    yield rbl, ctx
    ctx.close()


def _windows():
    starts = np.linspace(512, N - 1024, 24).astype(np.int64)
    return [(0, 512)] + [(int(s), int(s) + 512) for s in starts] + [(N - 517, N)]


def test_c5_spmm_sampled_rows(c5):
    rbl, ctx = c5
    assert ctx.spmm_kernel_for(B) == 5
    with pytest.raises(rbl.RBLError):          # the CSR is gone: only the band tiles remain
        ctx.get_matrix_csr()
    X = np.random.default_rng(7).standard_normal((N, B))
    log("X ready")
    Y = ctx.apply(X)
    log("A X on the device")
    aX = np.abs(X)
    for a, b in _windows():
        rp, col, val = rbl._lib.hashwindow_rows_host(N, HALFWIDTH, DENSITY, SEED, PLANT, a, b)
        As = sp.csr_matrix((val, col, rp), shape=(b - a, N))
        ref = As @ X
        bound = (abs(As) @ aX) * SPMM_TOL + 1e-300
        err = np.abs(Y[a:b] - ref)
        assert np.all(err <= bound), (a, float(np.max(err / bound)))
    log("sampled rows checked")


def test_c5_mixed_rbl_gpu_spilled(c5):
    rbl, ctx = c5
    ctx.set_option(rbl._lib.RBL_OPT_DEVICE_BLOCKS, DEVICE_BLOCKS)
    D, V, info = rbl.lanczos(ctx, K, B, seed=SEED + 2, check=True, ritz=True, basis_bits=32)
    log(f"mixed RBL_gpu: {info.iters} steps")
    assert info.converged and D.shape == (K,) and V.shape == (N, K)
    assert info.iters > DEVICE_BLOCKS          # the partial reorth and Ritz streamed spilled blocks
    assert np.all(np.diff(np.abs(D)) <= 0)     # P11
    assert 3900 < D[0] < 4100                  # the planted top of the spectrum
    Vp = np.zeros((N, B))
    Vp[:, :K] = V
    AV = ctx.apply(Vp)[:, :K]
    del Vp
    log("A V on the device")
    res = np.linalg.norm(AV - V * D, axis=0) / np.abs(D)
    assert res.max() < RES_TOL, res
    G = V.T @ V
    assert np.abs(G - np.eye(K)).max() < ORTH_TOL, np.abs(G - np.eye(K)).max()
    rq = np.einsum("ij,ij->j", V, AV) / np.einsum("ij,ij->j", V, V)
    assert np.all(np.abs(rq - D) <= RAYLEIGH_TOL * np.abs(D)), np.abs(rq - D) / np.abs(D)
    log("Ritz pairs checked")


def test_c5_deep_spill_bit_identical(c5):
    """The capacity regime at C5's n: 16 fixed steps with only DEVICE_BLOCKS slots in HBM (10 of
    the 16 fp32 blocks, 64 GB, in pinned host memory, streamed back over PCIe for every partial
    reorth) against the same 16 steps with the whole basis resident (109 GB of fp32 slots).  In
    the reference's block-MGS order (RBL_OPT_REORTH_ORDER = 1, RBL_gpu.jl:62-68) both apply the
    same kernels to the same blocks in the same order, so every A_i and B_{i+1} is the same bits."""
    rbl, ctx = c5
    steps = 16
    traces = []
    for device_blocks in (DEVICE_BLOCKS, 0):
        ctx.set_option(rbl._lib.RBL_OPT_REORTH_ORDER, 1)
        ctx.set_option(rbl._lib.RBL_OPT_DEVICE_BLOCKS, device_blocks)
        _, _, info = rbl.lanczos(ctx, K, B, seed=SEED + 4, check=False, max_steps=steps, trace=True,
                                 ritz=False, basis_bits=32)
        assert info.iters == steps and len(info.trace_A) == steps
        traces.append(info)
        log(f"{steps} steps, device blocks {device_blocks or 'all'}")
    ctx.set_option(rbl._lib.RBL_OPT_REORTH_ORDER, 0)
    spilled, resident = traces
    for a1, a2 in zip(spilled.trace_A + spilled.trace_B, resident.trace_A + resident.trace_B):
        assert np.all(np.isfinite(a1)) and np.array_equal(a1, a2)
