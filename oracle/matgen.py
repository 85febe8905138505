"""NumPy restatement of the seeded hash-window matrix generator — TEST INFRASTRUCTURE ONLY.

The synthetic inputs of SURVEY.md §8(d) (C1/C2/C4a) are defined by this generator; the HIP
library generates the same bits on the device (gen.hip) and on the host
(plan.cpp: rbl_hashwindow_rows_host).  Tests assert all three agree bit for bit.

Definition: entry (r, c), |r - c| <= W, r != c, exists iff u53(h(seed, min, max)) < p with
h = mix64(mix64(seed + lo) ^ hi); its value is 2 u - 1, u = u53(mix64(h ^ K)).  The diagonal
always exists with value 2u-1 (h(seed, r, r)) plus plant[l] at row l * floor(n / nplant).
"""
from __future__ import annotations

import numpy as np
import scipy.sparse as sp

_M = np.uint64(0xFFFFFFFFFFFFFFFF)
_K = np.uint64(0x5851F42D4C957F2D)


def mix64(z):
    z = np.asarray(z, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = z + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return z ^ (z >> np.uint64(31))


def pair_hash(seed, lo, hi):
    with np.errstate(over="ignore"):
        return mix64(mix64(np.uint64(seed) + np.asarray(lo).astype(np.uint64))
                     ^ np.asarray(hi).astype(np.uint64))


def u53(h):
    return (h >> np.uint64(11)).astype(np.float64) * 2.0 ** -53


def hashwindow_csr(n: int, W: int, p: float, seed: int, plant=None, row_begin=0, row_end=None):
    """Rows [row_begin, row_end) of the symmetric hash-window matrix as SciPy CSR (shape m x n)."""
    row_end = n if row_end is None else row_end
    rows = np.arange(row_begin, row_end, dtype=np.int64)
    d = np.arange(-W, W + 1, dtype=np.int64)
    R = np.repeat(rows, d.size)
    Cc = (rows[:, None] + d[None, :]).ravel()
    ok = (Cc >= 0) & (Cc < n)
    R, Cc = R[ok], Cc[ok]
    lo = np.minimum(R, Cc)
    hi = np.maximum(R, Cc)
    h = pair_hash(seed, lo, hi)
    diag = R == Cc
    keep = diag | (u53(h) < p)
    R, Cc, h, diag = R[keep], Cc[keep], h[keep], diag[keep]
    u = u53(mix64(h ^ _K))
    val = (u + u) - 1.0
    if plant is not None and len(plant):
        plant = np.asarray(plant, dtype=np.float64)
        stride = n // len(plant)
        pr = R[diag]
        add = np.zeros(pr.size)
        sel = (pr % stride == 0) & (pr // stride < len(plant))
        add[sel] = plant[pr[sel] // stride]
        val[np.flatnonzero(diag)] += add
    m = row_end - row_begin
    A = sp.csr_matrix((val, (R - row_begin, Cc)), shape=(m, n))
    A.sort_indices()
    return A


def hashwindow_csr_chunked(n: int, W: int, p: float, seed: int, plant=None, chunk: int = 200_000):
    """hashwindow_csr over all n rows built [chunk] rows at a time (the one-shot form needs ~10 GB
    per candidate array at n = 1e7): the same matrix bit for bit, int32 indices (nnz < 2^31)."""
    vals, cols, counts = [], [], []
    for r0 in range(0, n, chunk):
        A = hashwindow_csr(n, W, p, seed, plant, r0, min(n, r0 + chunk))
        vals.append(A.data)
        cols.append(A.indices.astype(np.int32))
        counts.append(np.diff(A.indptr))
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.concatenate(counts), out=rowptr[1:])
    val = np.concatenate(vals)
    del vals
    col = np.concatenate(cols)
    del cols
    assert rowptr[-1] < 2 ** 31
    return sp.csr_matrix((val, col, rowptr.astype(np.int32)), shape=(n, n))


_RMAT_K = np.uint64(0xD1B54A32D192ED03)


def rmat_draws(n: int, scale: int, edges: int, seed: int, a=0.57, b=0.19, c=0.19,
               edge_begin: int = 0, edge_end: int | None = None):
    """Kept R-MAT draws (r, c) in draw order (gen_rmat.hip: rmat_draw); draws
    [edge_begin, edge_end) of the `edges` (all by default), so large draws can be made in chunks."""
    edge_end = edges if edge_end is None else min(edge_end, edges)
    e = np.arange(edge_begin, edge_end, dtype=np.int64)
    edges = e.size
    s2 = np.uint64(seed) ^ _RMAT_K
    ab, abc = a + b, a + b + c
    r = np.zeros(edges, np.int64)
    cc = np.zeros(edges, np.int64)
    for lvl in range(scale):
        u = u53(pair_hash(s2, e, np.full(edges, lvl, np.int64)))
        bit = np.int64(1) << np.int64(scale - 1 - lvl)
        r |= np.where(u >= ab, bit, 0)
        cc |= np.where(((u >= a) & (u < ab)) | (u >= abc), bit, 0)
    keep = (r < n) & (cc < n) & (r != cc)
    return r[keep], cc[keep]


_RELABEL_K = 0x52454C4142454C31  # kernels.hpp kRelabelK ("RELABEL1")


def rmat_relabel(n: int, seed: int, idx, inverse=False):
    """RBL_OPT_RELABEL's permutation of the R-MAT vertex ids (gen_rmat.hip rmat_id): the Feistel
    bijection of scatter_perm under the key seed ^ kRelabelK."""
    return scatter_perm(n, int(np.uint64(seed) ^ np.uint64(_RELABEL_K)), idx, inverse)


def rmat_csr(n: int, scale: int, edges: int, seed: int, plant=None, row_begin=0, row_end=None,
             a=0.57, b=0.19, c=0.19, relabel=False):
    """Rows [row_begin, row_end) of the symmetric R-MAT matrix as SciPy CSR,
    restating gen_rmat.hip: both orientations of every kept draw (duplicates merged), the
    hash-window pair values off the diagonal, every diagonal entry with its hash value plus
    the planted spectrum.  relabel: P A P^T with vertex v at row / column rmat_relabel(v) (the
    values those of the original ids), as gen_rmat.hip with RBL_OPT_RELABEL = 1."""
    row_end = n if row_end is None else row_end
    r, cc = rmat_draws(n, scale, edges, seed, a, b, c)
    R = np.concatenate([r, cc, np.arange(n, dtype=np.int64)])
    C = np.concatenate([cc, r, np.arange(n, dtype=np.int64)])
    if relabel:
        Rn = rmat_relabel(n, seed, R)
        sel = (Rn >= row_begin) & (Rn < row_end)
        key = np.unique(Rn[sel] * np.int64(n) + rmat_relabel(n, seed, C[sel]))
        Rn, Cn = key // n, key % n
        R, C = rmat_relabel(n, seed, Rn, inverse=True), rmat_relabel(n, seed, Cn, inverse=True)
    else:
        sel = (R >= row_begin) & (R < row_end)
        key = np.unique(R[sel] * np.int64(n) + C[sel])
        R, C = key // n, key % n
        Rn, Cn = R, C
    lo, hi = np.minimum(R, C), np.maximum(R, C)
    u = u53(mix64(pair_hash(seed, lo, hi) ^ _K))
    val = (u + u) - 1.0
    if plant is not None and len(plant):
        plant = np.asarray(plant, dtype=np.float64)
        stride = n // len(plant)
        d = R == C
        sel2 = d & (R % stride == 0) & (R // stride < len(plant))
        val[sel2] += plant[R[sel2] // stride]
    m = row_end - row_begin
    A = sp.csr_matrix((val, (Rn - row_begin, Cn)), shape=(m, n))
    A.sort_indices()
    return A


def planted_spectrum(k: int, scale: float = 100.0):
    """Planted diagonal of SURVEY §8(d) C1: 2k entries at scale*(2k+1-l), l = 1..2k."""
    return np.array([scale * (2 * k + 1 - l) for l in range(1, 2 * k + 1)], dtype=np.float64)


def random_sym_csr(n: int = 10_000, density: float = 0.01, seed: int = 20261015, plant=None):
    """SURVEY §8(d) C1 as defined there: A = R + R^T, R with `density` nonzeros at uniformly
    random positions and N(0,1) values (numpy's PCG64 from `seed`), plus the planted diagonal at
    rows 0 .. len(plant) - 1 (the top of the spectrum, so the top k converge).  Unbanded: every
    row reaches the whole matrix (the GPU takes the segmented gather)."""
    rng = np.random.default_rng(seed)
    R = sp.random(n, n, density=density, format="csr", random_state=rng,
                  data_rvs=rng.standard_normal)
    A = (R + R.T).tocsr()
    if plant is not None:
        d = np.zeros(n)
        d[:len(plant)] = plant
        A = (A + sp.diags(d)).tocsr()
    A.sort_indices()
    A.eliminate_zeros()
    return A


_CIRC_K = np.uint64(0x9FB21C651E98DF25)
_SCATTER_K = np.uint64(0xA0761D6478BD642F)


def _feistel_half(n: int) -> int:
    h = 1
    while (1 << (2 * h)) < n:
        h += 1
    return h


def _feistel(x, key, half, inverse=False):
    """4-round Feistel network on 2*half-bit words (rbl_common.hpp scatter_round)."""
    mask = np.uint64((1 << half) - 1)
    L = x >> np.uint64(half)
    R = x & mask
    rounds = range(3, -1, -1) if inverse else range(4)
    for r in rounds:
        rk = key ^ (np.uint64(r) << np.uint64(56))
        if inverse:
            L, R = R ^ (mix64(rk ^ L) & mask), L
        else:
            L, R = R, L ^ (mix64(rk ^ R) & mask)
    return (L << np.uint64(half)) | R


def scatter_perm(n: int, seed: int, idx, inverse=False):
    """Seeded bijection of [0, n) (gen.hip scatter / scatter_inv): the Feistel network above on
    the smallest even bit width covering n, cycle-walked back into [0, n)."""
    half = _feistel_half(n)
    key = mix64(np.uint64(seed) ^ _SCATTER_K)
    x = np.asarray(idx, dtype=np.uint64).copy()
    todo = np.ones(x.shape, bool)
    while todo.any():
        x[todo] = _feistel(x[todo], key, half, inverse)
        todo = x >= np.uint64(n)
    return x.astype(np.int64)
G3_CIRCUIT_N = 1_585_478          # SuiteSparse G3_circuit (BASELINE config 3): n
G3_CIRCUIT_NNZ = 7_660_826        #   and stored nonzeros, both triangles (4.83 per row)


def circuit_like_csr(n: int = G3_CIRCUIT_N, seed: int = 20261015, plant=None, width: int = 1259,
                     p_edge: float = 0.95873):
    """A circuit-like SPD matrix of G3_circuit's shape (BASELINE config 3; the real .mtx is not
    in this image and is not fetched): a weighted graph Laplacian on a 5-point stencil over
    rows of `width` nodes (nodes i, i+1 in one row; i, i+width), each edge kept iff
    u53(h(seed, lo, hi)) < p_edge (so ~4.83 nonzeros per row at the defaults, like
    G3_circuit's 7.66 M over 1.59 M rows), weight 0.5 + u53(mix64(h ^ K)); diagonal = the row's
    weight sum + 0.01 (+ plant[l] at node l * floor(n / len(plant))), summed in the order
    0.01, right, down, left, up neighbour.  Then a seeded symmetric permutation (scatter_perm:
    a Feistel bijection, so the device generator rbl_gen_matrix_circuit builds the same bits
    row by row) scatters the pattern over the whole index range, as circuit matrices are: no
    band, so the gather SpMM runs, not the band tiles.  Returns SciPy CSR (n x n)."""
    i = np.arange(n, dtype=np.int64)
    lo_h = i[(i % width) != width - 1]
    lo_h = lo_h[lo_h + 1 < n]
    lo_v = i[i + width < n]
    lo = np.concatenate([lo_h, lo_v])
    hi = np.concatenate([lo_h + 1, lo_v + width])
    h = pair_hash(seed, lo, hi)
    keep = u53(h) < p_edge
    lo, hi, h = lo[keep], hi[keep], h[keep]
    w = 0.5 + u53(mix64(h ^ _CIRC_K))
    diag = np.full(n, 0.01)
    np.add.at(diag, lo, w)
    np.add.at(diag, hi, w)
    if plant is not None and len(plant):
        plant = np.asarray(plant, dtype=np.float64)
        stride = n // len(plant)
        if stride > 0:  # (n < len(plant): no plant, as the device generator)
            diag[np.arange(len(plant)) * stride] += plant
    # seeded symmetric permutation (node i -> perm[i]): a hash bijection the device generator
    # (gen.hip k_circ_fill) computes per row
    perm = scatter_perm(n, seed, np.arange(n, dtype=np.int64))
    R = np.concatenate([perm[lo], perm[hi], perm])
    C = np.concatenate([perm[hi], perm[lo], perm])
    V = np.concatenate([-w, -w, diag])
    A = sp.csr_matrix((V, (R, C)), shape=(n, n))
    A.sort_indices()
    return A
