#!/usr/bin/env python3
"""Full-size eigenvalue fixtures for BASELINE configs 2 and 3 (committed; regenerate from the
repo root with ``python tests/golden/make_fullsize.py [c2|c3|c4b|c4a]``; ~2-10 min each on 8
cores, c4a ~30 min and ~45 GB of host memory).

The expected outputs come from the oracle (oracle/rbl_oracle.py: the CPU restatement of
RBL.jl:74-142 with the GPU driver's bounds, RBL_gpu.jl:134-219, and the HIP path's choices —
positive-diagonal QR, block-CGS partial reorth), run here on the configs' own sizes.
Fixtures are data only: the generator parameters, Omega's seed, and the outputs.

  golden_c2.npz  C2: n = 1e6 hash-window (half-width 32, density 0.7734: ~50 nnz/row),
                 planted top spectrum, b = 16, k = 20.
  golden_c3.npz  C3-shaped: matgen.circuit_like_csr — n = 1,585,478 and 7.66 M nonzeros like
                 SuiteSparse G3_circuit (BASELINE config 3; the real file is not in this image
                 and is not fetched), SPD weighted Laplacian, scattered by a symmetric
                 permutation (no band), planted top spectrum; b = 16, k = 20.

  golden_c4b.npz BASELINE config 4's R-MAT pattern at n = 1e6: matgen.rmat_csr with
                 (a,b,c,d) = (0.57,0.19,0.19,0.05), scale 20, 0.66 n x 100 draws (the bench's
                 C4b draw density: ~100 nnz/row after symmetrising and merging; hub rows of
                 ~1e5 nonzeros, so the segmented gather splits them), planted top spectrum;
                 b = 32, k = 20.  The device generator (gen_rmat.hip) builds the same bits.

  golden_c4a.npz BASELINE's headline config at FULL size (the bench's C4a workload): n = 1e7
                 hash-window (half-width 64, density 0.7734: ~100 nnz/row, 0.9999 G nonzeros),
                 planted top spectrum, b = 32, k = 20.  Built in row chunks; the partial
                 reorth is the same block CGS evaluated block by block (reorth_mode
                 "cgs_blocked") so the oracle fits the 62 GB container.

Each holds D (k, descending |lambda|), the iteration count, and per Ritz vector its 16
largest-magnitude entries (row ids + values) — enough to compare vectors up to sign without
storing n x k numbers — the residual norms ||A v - lambda v|| / |lambda|, and the per-step
block trace (trace_A[i] = A_{i+1}, trace_B[i] = B_{i+2}: RBL_gpu.jl:153-161 then :176-184 of
every loop step), so the block-step semantics are pinned at full size, not only their end
product (round 6 regenerated c4a and c4b_full with the traces; D and iters are unchanged).
"""
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import matgen  # noqa: E402
from oracle import rbl_oracle as o  # noqa: E402

C2 = dict(n=1_000_000, halfwidth=32, density=0.7734, seed=20261015, b=16, k=20, omega_seed=2)
C3 = dict(n=matgen.G3_CIRCUIT_N, seed=20261015, b=16, k=20, omega_seed=3)
C4B = dict(n=1_000_000, scale=20, edges=66_000_000, seed=20261015, b=32, k=20, omega_seed=4)
# BASELINE's headline config (the bench's C4a workload): n = 1e7, half-width 64, ~100 nnz/row
C4A = dict(n=10_000_000, halfwidth=64, density=0.7734, seed=20261015, b=32, k=20, omega_seed=5)
TOP = 16


def c2_matrix():
    return matgen.hashwindow_csr(C2["n"], C2["halfwidth"], C2["density"], C2["seed"],
                                 matgen.planted_spectrum(C2["k"]))


def c3_matrix():
    return matgen.circuit_like_csr(C3["n"], C3["seed"], matgen.planted_spectrum(C3["k"]))


def c4b_matrix():
    return matgen.rmat_csr(C4B["n"], C4B["scale"], C4B["edges"], C4B["seed"],
                           matgen.planted_spectrum(C4B["k"]))


def c4a_matrix(chunk=200_000):
    """C4a's CSR built in row chunks (matgen.hashwindow_csr_chunked: the same matrix bit for bit)."""
    return matgen.hashwindow_csr_chunked(C4A["n"], C4A["halfwidth"], C4A["density"], C4A["seed"],
                                         matgen.planted_spectrum(C4A["k"]), chunk)


# C4b at BASELINE's full size (the bench's sub-record, as drawn: RBL_OPT_RELABEL 0)
C4B_FULL = dict(n=10_000_000, scale=24, edges=660_000_000, seed=20261015, b=32, k=20, omega_seed=6)


def c4b_full_matrix(edge_chunk=20_000_000, row_chunk=1_000_000):
    """matgen.rmat_csr (relabel off) built in chunks: the kept draws made [edge_chunk] at a time
    and kept as int32 (n < 2^31), then each row range's keys (both orientations of every draw
    plus the diagonal) merged with np.unique, values and plant exactly as rmat_csr — the same
    matrix bit for bit (checked against rmat_csr at small n by test_oracle), in ~1/5 of the
    memory.  int32 indices: nnz < 2^31."""
    import scipy.sparse as sp
    cfg = C4B_FULL
    n, scale, edges, seed = cfg["n"], cfg["scale"], cfg["edges"], cfg["seed"]
    return rmat_csr_chunked(n, scale, edges, seed, matgen.planted_spectrum(cfg["k"]),
                            edge_chunk, row_chunk)


def rmat_csr_chunked(n, scale, edges, seed, plant, edge_chunk, row_chunk):
    import scipy.sparse as sp
    rs, cs = [], []
    for e0 in range(0, edges, edge_chunk):
        r, c = matgen.rmat_draws(n, scale, edges, seed, edge_begin=e0, edge_end=e0 + edge_chunk)
        rs.append(r.astype(np.int32))
        cs.append(c.astype(np.int32))
    r = np.concatenate(rs); del rs
    c = np.concatenate(cs); del cs
    plant = np.asarray(plant, dtype=np.float64)
    stride = n // len(plant)
    vals, cols, counts = [], [], []
    for a in range(0, n, row_chunk):
        b = min(n, a + row_chunk)
        s1 = (r >= a) & (r < b)
        s2 = (c >= a) & (c < b)
        R = np.concatenate([r[s1], c[s2]]).astype(np.int64)
        C = np.concatenate([c[s1], r[s2]]).astype(np.int64)
        del s1, s2
        d = np.arange(a, b, dtype=np.int64)
        key = np.unique(np.concatenate([R * np.int64(n) + C, d * np.int64(n) + d]))
        del R, C
        R, C = key // n, key % n
        del key
        lo, hi = np.minimum(R, C), np.maximum(R, C)
        u = matgen.u53(matgen.mix64(matgen.pair_hash(seed, lo, hi) ^ matgen._K))
        val = (u + u) - 1.0
        dg = R == C
        sel2 = dg & (R % stride == 0) & (R // stride < len(plant))
        val[sel2] += plant[R[sel2] // stride]
        vals.append(val)
        cols.append(C.astype(np.int32))
        counts.append(np.bincount(R - a, minlength=b - a))
    del r, c
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.concatenate(counts), out=rowptr[1:])
    val = np.concatenate(vals); del vals
    col = np.concatenate(cols); del cols
    assert rowptr[-1] < 2 ** 31
    return sp.csr_matrix((val, col, rowptr.astype(np.int32)), shape=(n, n))


def omega_for(cfg):
    return np.random.default_rng(cfg["omega_seed"]).standard_normal((cfg["n"], cfg["b"]))


def run(name, cfg, A, reorth_mode="cgs"):
    t0 = time.perf_counter()
    res = o.RBL_gpu_semantics(A, cfg["k"], cfg["b"], omega=omega_for(cfg), qr_mode="posdiag",
                              reorth_mode=reorth_mode, trace=True)
    dt = time.perf_counter() - t0
    assert res.converged, name
    V = res.V
    idx = np.argsort(-np.abs(V), axis=0)[:TOP]            # TOP x k row ids
    vals = np.take_along_axis(V, idx, axis=0)
    r = np.linalg.norm(A @ V - V * res.D, axis=0) / np.abs(res.D)
    out = os.path.join(HERE, f"golden_{name}.npz")
    import resource
    peak_rss_gb = resource.getrusage(resource.RUSAGE_SELF).ru_maxrss / 2 ** 20
    np.savez_compressed(out, D=res.D, iters=res.iters, top_idx=idx.astype(np.int64), top_val=vals,
                        residual=r, nnz=A.nnz, oracle_seconds=dt, peak_rss_gb=peak_rss_gb,
                        reorth_mode=reorth_mode,
                        # per block step i (rbl_start's step 1 first): A_i and B_{i+1}, b x b each
                        # (positive-diagonal R, so B needs no sign normalisation)
                        trace_A=np.array(res.trace["A"]), trace_B=np.array(res.trace["B"]),
                        **{f"cfg_{key}": v for key, v in cfg.items()})
    print(f"{name}: n={A.shape[0]} nnz={A.nnz} iters={res.iters} D[:3]={res.D[:3]} "
          f"max residual={r.max():.2e} ({dt:.1f} s, peak RSS {peak_rss_gb:.1f} GB) -> {out}",
          flush=True)


def main(which):
    if "c2" in which:
        run("c2", C2, c2_matrix())
    if "c3" in which:
        run("c3", C3, c3_matrix())
    if "c4b" in which:
        run("c4b", C4B, c4b_matrix())
    if "c4b_full" in which:
        import resource
        # a MemoryError instead of the OOM killer if the estimate (~55 GB) is wrong
        lim = int(float(os.environ.get("RBL_FIXTURE_MEM_GB", "58")) * 2 ** 30)
        resource.setrlimit(resource.RLIMIT_DATA, (lim, lim))
        t0 = time.perf_counter()
        A = c4b_full_matrix()
        print(f"c4b_full: matrix {A.nnz} nonzeros in {time.perf_counter() - t0:.1f} s", flush=True)
        run("c4b_full", C4B_FULL, A, reorth_mode="cgs_blocked")
    if "c4a" in which:
        t0 = time.perf_counter()
        A = c4a_matrix()
        print(f"c4a: matrix {A.nnz} nonzeros in {time.perf_counter() - t0:.1f} s", flush=True)
        # block CGS evaluated block by block: no n x (i-2)b copy of the basis (62 GB container)
        run("c4a", C4A, A, reorth_mode="cgs_blocked")


if __name__ == "__main__":
    main(sys.argv[1:] or ["c2", "c3", "c4b"])
