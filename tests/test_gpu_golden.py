"""GPU: the HIP path through the C-ABI against the committed golden fixtures (no live oracle).

Tolerances (north star: eigenvalue error < 1e-10): D within 1e-10 relative, Ritz vectors
1 - |v.v'| < 1e-8 and residual ||Av - lambda v|| / |lambda| < 1e-7, per-step A_i / B_i within
1e-9 relative (CholQR and the posdiag oracle share the sign convention, P4); device generator
bit-exact.
"""
import os

import numpy as np
import pytest
import scipy.sparse as sp

pytestmark = pytest.mark.gpu

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def rbl():
    import rbl as _r
    return _r


def c1():
    z = np.load(os.path.join(G, "golden_c1.npz"))
    n = int(z["n"])
    return z, sp.csr_matrix((z["data"], z["indices"], z["indptr"]), shape=(n, n))


@pytest.mark.parametrize("order", [0, 1])
def test_gpu_reproduces_c1_golden(rbl, order):
    z, A = c1()
    k, b = int(z["k"]), int(z["b"])
    D, V, info = rbl.RBL_gpu(A, k, b, omega=z["omega"], reorth_order=order, return_info=True)
    assert info.converged and info.iters == int(z["iters"])
    assert np.max(np.abs(D - z["D"]) / np.abs(z["D"])) < 1e-10
    dots = np.abs(np.sum(V * z["V"], axis=0))
    assert np.all(1 - dots < 1e-8), dots
    res = np.linalg.norm(A @ V - V * D[None, :], axis=0) / np.abs(D)
    assert np.all(res < 1e-7)


def test_gpu_trace_matches_c1_golden(rbl):
    z, A = c1()
    b = int(z["b"])
    with rbl.Context(0) as ctx:
        ctx.set_matrix(A)
        _, _, info = rbl.lanczos(ctx, int(z["k"]), b, omega=z["omega"], check=False,
                                 max_steps=8, trace=True, ritz=False)
    for a, ag in zip(info.trace_A, z["trace_A"]):
        assert np.abs(a - ag).max() <= 1e-9 * np.abs(ag).max()
    for bb, bg in zip(info.trace_B, z["trace_B"]):
        assert np.abs(bb - bg).max() <= 1e-9 * np.abs(bg).max()


def test_device_generator_matches_golden_rows(rbl):
    z = np.load(os.path.join(G, "golden_hashwindow.npz"))
    n, W, p, seed, plant = int(z["n"]), int(z["W"]), float(z["p"]), int(z["seed"]), z["plant"]
    with rbl.Context(0) as ctx:
        ctx.gen_hashwindow(n, W, p, seed, plant)
        rp, col, val = ctx.get_matrix_csr()
    for tag in ("head", "tail"):
        r0, r1 = (int(x) for x in z[f"{tag}_rows"])
        e0, e1 = rp[r0], rp[r1]
        assert np.array_equal(rp[r0:r1 + 1] - e0, z[f"{tag}_indptr"])
        assert np.array_equal(col[e0:e1].astype(np.int64), z[f"{tag}_indices"])
        assert np.array_equal(val[e0:e1].view(np.uint64), z[f"{tag}_data"].view(np.uint64))
