#!/usr/bin/env python3
"""Which block steps take CholQR's shifted third pass, and how far the step traces of the
local-reorth Gram formed inside the QR (RBL_OPT_FUSE 3) are from the separate Gram (1) there —
on diagonal matrices whose spectrum is m clusters of width w, so the Krylov blocks become
nearly dependent after ~m/b steps.  Prints per step: status (1 = shifted), B's norm, and the
relative A_i / B_{i+1} differences.  (Diagnostic for the test of k_cloc_rinv.)"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-randomized-block-lanczos_amd")]
import numpy as np  # noqa: E402
import scipy.sparse as sp  # noqa: E402
import rbl  # noqa: E402
from rbl import _lib  # noqa: E402


def run(A, b, fuse, steps, omega):
    with rbl.Context(0) as ctx:
        ctx.set_option(_lib.RBL_OPT_FUSE, fuse)
        ctx.set_matrix(A)
        ctx.start(b, steps, omega=omega)
        for i in range(1, steps + 1):
            ctx.step_async(i, i >= 2 and i % 2 == 0)
        return ctx.fetch(1, steps + 1)


for b in (16, 32):
    for m, w in ((3 * b + 5, 1e-9), (4 * b + 3, 1e-7), (2 * b + 1, 1e-5)):
        n = 3000
        rng = np.random.default_rng(m)
        vals = np.linspace(1.0, 10.0, m)
        lam = vals[np.arange(n) % m] + w * rng.standard_normal(n)
        A = sp.diags(lam).tocsc()
        omega = rng.standard_normal((n, b))
        steps = 10
        r1 = run(A, b, 1, steps, omega)
        r3 = run(A, b, 3, steps, omega)
        print(f"b={b} clusters={m} width={w:g}")
        for i, ((A1, B1, s1), (A3, B3, s3)) in enumerate(zip(r1, r3), start=1):
            da = np.abs(A3 - A1).max() / np.abs(A1).max()
            db = np.abs(B3 - B1).max() / max(np.abs(B1).max(), 1e-300)
            print(f"  step {i:2d} st={s1},{s3} |B|={np.abs(B1).max():9.2e} dA={da:8.1e} dB={db:8.1e}")
