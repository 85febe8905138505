"""GPU: the host-spill Krylov basis (RBL_OPT_DEVICE_BLOCKS) — the reference's hybrid buffer
(RBL_gpu.jl:24-27 gpu_buffer_size, 59-81 hybrid_part_reorth!, 106-132 recover_eigvec): the
first G-2 blocks stay in HBM, the two newest in working slots, every older block in pinned host
memory, streamed back for partial reorth and the Ritz vectors.

Tolerances: with the reference's block-MGS order (RBL_OPT_REORTH_ORDER = 1) the spilled run
applies the same operations in the same order as the resident one: per-step A_i within 1e-12
relative.  With the default block CGS the resident part is batched and the spilled part
applied block by block (the reference's order): eigenvalues within 1e-10 of the resident run
and of the oracle, Ritz vectors 1 - |v.v'| < 1e-8, per-step A_i within 1e-9."""
import numpy as np
import pytest

from oracle import matgen
from oracle import rbl_oracle as o

pytestmark = pytest.mark.gpu

K, B = 10, 16


@pytest.fixture(scope="module")
def rbl():
    import rbl as _r
    return _r


@pytest.fixture(scope="module")
def problem():
    A = matgen.hashwindow_csr(6000, 48, 0.5, 21, matgen.planted_spectrum(K))
    omega = np.random.default_rng(5).standard_normal((A.shape[0], B))
    return A, omega


def _run(rbl, A, omega, device_blocks, order=0, steps=None, check=True):
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        ctx.set_option(rbl._lib.RBL_OPT_REORTH_ORDER, order)
        ctx.set_option(rbl._lib.RBL_OPT_DEVICE_BLOCKS, device_blocks)
        D, V, info = rbl.lanczos(ctx, K, B, omega=omega, check=check, max_steps=steps, trace=True)
        blocks = [ctx.get_block(j) for j in range(1, ctx.num_blocks() + 1)]
    return D, V, info, blocks


@pytest.mark.parametrize("G", [3, 4, 7])
def test_spill_mgs_order_matches_resident(rbl, problem, G):
    A, omega = problem
    _, _, i1, b1 = _run(rbl, A, omega, 0, order=1, steps=14, check=False)
    _, _, i2, b2 = _run(rbl, A, omega, G, order=1, steps=14, check=False)
    for a1, a2 in zip(i1.trace_A, i2.trace_A):
        assert np.abs(a1 - a2).max() <= 1e-12 * np.abs(a1).max()
    for q1, q2 in zip(b1, b2):          # every block, spilled ones read back from the host
        assert np.abs(q1 - q2).max() <= 1e-12


@pytest.mark.parametrize("G", [3, 5])
def test_spill_cgs_full_run(rbl, problem, G):
    A, omega = problem
    D1, V1, i1, _ = _run(rbl, A, omega, 0)
    D2, V2, i2, _ = _run(rbl, A, omega, G)
    assert i1.converged and i2.converged and i2.iters == i1.iters
    assert np.max(np.abs(D2 - D1) / np.abs(D1)) < 1e-10
    assert np.all(1 - np.abs(np.sum(V1 * V2, axis=0)) < 1e-8)
    for a1, a2 in zip(i1.trace_A, i2.trace_A):
        assert np.abs(a1 - a2).max() <= 1e-9 * np.abs(a1).max()
    ref = o.RBL_gpu_semantics(A, K, B, omega=omega, qr_mode="posdiag", reorth_mode="cgs")
    assert np.max(np.abs(D2 - ref.D) / np.abs(ref.D)) < 1e-10
    res = np.linalg.norm(A @ V2 - V2 * D2, axis=0) / np.abs(D2)
    assert res.max() < 1e-7


def test_spill_auto_and_guards(rbl, problem):
    A, omega = problem
    D1, _, _, _ = _run(rbl, A, omega, 0)
    Da, _, _, _ = _run(rbl, A, omega, -1)        # everything fits: no spill, same bits
    assert np.array_equal(D1, Da)
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        with pytest.raises(rbl.RBLError):
            ctx.set_option(rbl._lib.RBL_OPT_DEVICE_BLOCKS, 2)
        ctx.set_option(rbl._lib.RBL_OPT_DEVICE_BLOCKS, 3)
        ctx.start(B, 10, omega=omega)
        for i in range(1, 6):
            ctx.step(i, i % 2 == 0)
        with pytest.raises(rbl.RBLError):
            ctx.restart(5, np.eye(5 * B)[:, :B].copy(order="F"))


# ---- the fp32 basis spilled (the reference's hybrid buffer is typed FLOAT: RBL_gpu.jl:59-81,
# 95-104 with FLOAT = Float32) ----------------------------------------------------------------
def _run32(rbl, A, omega, device_blocks, order=0, steps=None, check=True, k=K):
    b = omega.shape[1]
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        ctx.set_option(rbl._lib.RBL_OPT_REORTH_ORDER, order)
        ctx.set_option(rbl._lib.RBL_OPT_DEVICE_BLOCKS, device_blocks)
        D, V, info = rbl.lanczos(ctx, k, b, omega=omega, check=check, max_steps=steps,
                                 trace=True, basis_bits=32)
        blocks = [ctx.get_block(j) for j in range(1, ctx.num_blocks() + 1)]
    return D, V, info, blocks


@pytest.mark.parametrize("G,b", [(3, 16), (6, 32)])
def test_spill_fp32_mgs_order_bit_identical(rbl, G, b):
    """Block-MGS order: the resident run applies each block's Gram + update one at a time, the
    spilled run the same kernels on the block staged back from pinned memory: same bits."""
    A = matgen.hashwindow_csr(6000, 64, 0.7734, 21, matgen.planted_spectrum(K))
    omega = np.random.default_rng(5).standard_normal((A.shape[0], b))
    _, _, i1, b1 = _run32(rbl, A, omega, 0, order=1, steps=14, check=False)
    _, _, i2, b2 = _run32(rbl, A, omega, G, order=1, steps=14, check=False)
    for a1, a2 in zip(i1.trace_A + i1.trace_B, i2.trace_A + i2.trace_B):
        assert np.array_equal(a1, a2)
    for q1, q2 in zip(b1, b2):          # spilled blocks read back from the host
        assert np.array_equal(q1, q2)
        assert np.array_equal(q2, q2.astype(np.float32).astype(np.float64))


@pytest.mark.parametrize("G", [3, 5])
def test_spill_fp32_cgs_full_run(rbl, problem, G):
    """Default block CGS: resident part batched, spilled part block by block; eigenvalues vs
    the resident fp32 run and the mixed-mode oracle within the fp32-basis tolerance (1e-7)."""
    A, omega = problem
    D1, V1, i1, _ = _run32(rbl, A, omega, 0)
    D2, V2, i2, _ = _run32(rbl, A, omega, G)
    assert i1.converged and i2.converged and i2.iters == i1.iters
    assert np.max(np.abs(D2 - D1) / np.abs(D1)) < 1e-7
    ref = o.RBL_gpu_mixed(A, K, B, omega=omega, reorth_mode="cgs")
    assert np.max(np.abs(D2 - ref.D) / np.abs(ref.D)) < 1e-7
    res = np.linalg.norm(A @ V2 - V2 * D2, axis=0) / np.abs(D2)
    assert res.max() < 1e-5
    assert np.all(1 - np.abs(np.sum(V1 * V2, axis=0)) < 1e-6)
