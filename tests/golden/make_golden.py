#!/usr/bin/env python3
"""Regenerate the golden fixtures in tests/golden/ (committed; run from the repo root:
``python tests/golden/make_golden.py``).

The reference (Julia) cannot run in this container (no julia toolchain), so the
expected outputs come from the CPU restatement in oracle/ — which is itself pinned by the
reference's known-answer suites (Julia/Unit Testing/test.jl:16-50, *_dec.jl), whose expected
eigenvalues are stored here too.  Fixtures are data only (inputs + expected outputs).

  golden_c1.npz          C1-shaped case reduced to n=1200: A = R + R^T, R 1 %
                         density N(0,1), planted diagonal 100(2k+1-l), k=10, b=8, Omega.
                         Expected: D, V, per-step A_i / B_i (first 8 steps), iteration count —
                         GPU semantics (RBL_gpu.jl, kryl 1200) with positive-diagonal QR and
                         block-CGS partial reorth (the HIP path's choices), plus D under the
                         reference's own choices (Householder QR, ascending-j block MGS).
  golden_hashwindow.npz  rows [0,64) and [n-64,n) of the seeded hash-window generator
                         (the C2/C4a input family) — bit-exact for numpy / C++ host / device.
  golden_known_answer.npz  expected eigenvalues of the reference's three known-answer suites
                         (k=5, b=5) and the oracle's D on them.
"""
import os
import sys

import numpy as np
import scipy.sparse as sp

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import matgen  # noqa: E402
from oracle import rbl_oracle as o  # noqa: E402

C1_N, C1_K, C1_B, C1_SEED = 1200, 10, 8, 20261015
HW = dict(n=4096, W=24, p=0.45, seed=20261015, nplant=6)


def c1_matrix(n=C1_N, k=C1_K, seed=C1_SEED):
    rng = np.random.default_rng(seed)
    R = sp.random(n, n, density=0.01, random_state=rng, data_rvs=rng.standard_normal,
                  format="csr")
    plant = np.zeros(n)
    stride = n // (2 * k)
    for l in range(1, 2 * k + 1):
        plant[(l - 1) * stride] = 100.0 * (2 * k + 1 - l)
    A = sp.csr_matrix(R + R.T + sp.diags(plant))
    A.sort_indices()
    return A


def main():
    # ---- C1 ------------------------------------------------------------------------------
    A = c1_matrix()
    omega = np.random.default_rng(1).standard_normal((C1_N, C1_B))
    res = o.RBL_gpu_semantics(A, C1_K, C1_B, omega=omega, qr_mode="posdiag", reorth_mode="cgs",
                              trace=True)
    assert res.converged
    tr = o.RBL_gpu_semantics(A, C1_K, C1_B, omega=omega, qr_mode="posdiag", reorth_mode="cgs",
                             check=False, max_steps=8, trace=True).trace
    ref = o.RBL_gpu_semantics(A, C1_K, C1_B, omega=omega)   # Householder + block MGS
    np.savez_compressed(
        os.path.join(HERE, "golden_c1.npz"),
        n=C1_N, k=C1_K, b=C1_B, indptr=A.indptr.astype(np.int64),
        indices=A.indices.astype(np.int32), data=A.data, omega=omega,
        D=res.D, V=res.V, iters=res.iters, trace_A=np.stack(tr["A"]), trace_B=np.stack(tr["B"]),
        D_reference_choices=ref.D)
    # ---- hash-window generator rows -------------------------------------------------------
    n, W, p, seed = HW["n"], HW["W"], HW["p"], HW["seed"]
    plant = matgen.planted_spectrum(HW["nplant"] // 2)
    out = dict(n=n, W=W, p=p, seed=seed, plant=plant)
    for tag, (r0, r1) in {"head": (0, 64), "tail": (n - 64, n)}.items():
        M = matgen.hashwindow_csr(n, W, p, seed, plant, r0, r1)
        out[f"{tag}_rows"] = np.array([r0, r1])
        out[f"{tag}_indptr"] = M.indptr.astype(np.int64)
        out[f"{tag}_indices"] = M.indices.astype(np.int64)
        out[f"{tag}_data"] = M.data
    np.savez_compressed(os.path.join(HERE, "golden_hashwindow.npz"), **out)
    # ---- known-answer suites ----------------------------------------------------------------
    ka = {}
    for name, (gen, ns, k, b) in o.KNOWN_ANSWER_SUITES.items():
        for nn in ns:
            Am, eig = gen(nn, k)
            r = o.RBL(Am, k, b, seed=0)
            ka[f"{name}_{nn}_expected"] = eig
            ka[f"{name}_{nn}_oracle"] = r.D
    np.savez_compressed(os.path.join(HERE, "golden_known_answer.npz"), **ka)
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)), "bytes")


if __name__ == "__main__":
    main()
