"""Dump eigenvalues and the A_i/B_i trace of short runs (b = 16, 32; ragged n) with whichever
library RBL_LIB names, or compare two dumps bit for bit:
  python tools/r03_bitcmp.py dump out.npz
  python tools/r03_bitcmp.py cmp a.npz b.npz"""
import sys

import numpy as np

if sys.argv[1] == "cmp":
    a, b = np.load(sys.argv[2]), np.load(sys.argv[3])
    bad = [k for k in a.files if not np.array_equal(a[k], b[k])]  # float arrays only
    print("bit-identical" if not bad else f"DIFFER: {bad}")
    sys.exit(1 if bad else 0)

import os
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "gpu-randomized-block-lanczos_amd"))
import scipy.sparse as sp
import rbl

out = {}
for n in (3001, 20000):
    R = sp.random(n, n, density=min(0.004, 40.0 / n), random_state=5, format="csr")
    A = (R + R.T + sp.diags(np.linspace(1.0, 3.0, n))).tocsr()
    for b in (16, 32):
        omega = np.random.default_rng(b).standard_normal((n, b))
        with rbl.Context(0) as ctx:
            ctx.set_matrix(A)
            D, V, info = rbl.lanczos(ctx, 10, b, omega=omega, max_steps=14, trace=True)
            blk = np.stack([ctx.get_block(j) for j in range(1, min(ctx.num_blocks(), 8) + 1)])
        out[f"D_{n}_{b}"] = np.asarray(D)
        out[f"V_{n}_{b}"] = np.asarray(V, dtype=np.float64)
        out[f"Q_{n}_{b}"] = blk
        out[f"A_{n}_{b}"] = np.concatenate([np.ravel(x) for x in info.trace_A])
        out[f"B_{n}_{b}"] = np.concatenate([np.ravel(x) for x in info.trace_B])
        assert D.size and V is not None and blk.size, "nothing to compare"
np.savez(sys.argv[2], **out)
print("dumped", sys.argv[2], len(out))
