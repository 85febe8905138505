// gen.hip — device-side data preparation: the seeded hash-window matrix,
// the counter-based N(0,1) start block (replaces CUDA.randn, RBL_gpu.jl:213), per-tile
// column footprints for the LDS-window SpMM, and boundary layout transposes.
#include "kernels.hpp"

namespace rbl {

__global__ void k_hw_count(int64_t n, int64_t W, double p, uint64_t seed, int64_t r0, int64_t r1,
                           int32_t* counts) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = r0 + i;
  if (r >= r1) return;
  const int64_t lo = r - W < 0 ? 0 : r - W;
  const int64_t hi = r + W > n - 1 ? n - 1 : r + W;
  int cnt = 1;  // diagonal
  for (int64_t c = lo; c <= hi; ++c) {
    if (c == r) continue;
    const int64_t a = c < r ? c : r, bb = c < r ? r : c;
    cnt += hw_present(seed, a, bb, p) ? 1 : 0;
  }
  counts[i] = cnt;
}

__global__ void k_hw_fill(int64_t n, int64_t W, double p, uint64_t seed, int64_t r0, int64_t r1,
                          const int64_t* __restrict__ rowptr, int nplant,
                          const double* __restrict__ plant, int32_t* col, double* val) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = r0 + i;
  if (r >= r1) return;
  const int64_t lo = r - W < 0 ? 0 : r - W;
  const int64_t hi = r + W > n - 1 ? n - 1 : r + W;
  int64_t e = rowptr[i];
  const int64_t stride = nplant > 0 ? n / nplant : 0;
  for (int64_t c = lo; c <= hi; ++c) {
    if (c == r) {
      double d = hw_value(seed, r, r);
      if (stride > 0 && r % stride == 0 && r / stride < nplant) d += plant[r / stride];
      col[e] = (int32_t)c;
      val[e] = d;
      ++e;
      continue;
    }
    const int64_t a = c < r ? c : r, bb = c < r ? r : c;
    if (hw_present(seed, a, bb, p)) {
      col[e] = (int32_t)c;
      val[e] = hw_value(seed, a, bb);
      ++e;
    }
  }
}

void hw_count(int64_t n, int64_t W, double p, uint64_t seed, int64_t r0, int64_t r1,
              int32_t* counts, hipStream_t s) {
  const int64_t m = r1 - r0;
  if (m <= 0) return;
  hipLaunchKernelGGL(k_hw_count, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, n, W, p,
                     seed, r0, r1, counts);
}

void hw_fill(int64_t n, int64_t W, double p, uint64_t seed, int64_t r0, int64_t r1,
             const int64_t* rowptr, int nplant, const double* plant_dev, int32_t* col,
             double* val, hipStream_t s) {
  const int64_t m = r1 - r0;
  if (m <= 0) return;
  hipLaunchKernelGGL(k_hw_fill, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, n, W, p, seed,
                     r0, r1, rowptr, nplant, plant_dev, col, val);
}

// ---- circuit-like SPD matrix of G3_circuit's shape (BASELINE config 3; oracle/matgen.py
// circuit_like_csr): a weighted Laplacian on a 5-point stencil over rows of `width` nodes, each
// edge (lo, hi) kept iff u53(h) < p_edge (h = pair_hash(seed, lo, hi)), weight
// 0.5 + u53(mix64(h ^ K)); diagonal 0.01 + the kept weights in the order right, down, left, up
// (+ plant[l] at node l * floor(n / nplant)); node i becomes row / column scatter(i).  Row r of
// the result is node scatter_inv(r): at most 5 nonzeros, columns sorted in registers.
constexpr uint64_t kCircK = 0x9FB21C651E98DF25ull;

struct CircNb {
  int64_t node[4];
  double w[4];
  int cnt;
};

__device__ inline CircNb circ_neighbours(int64_t i, int64_t n, int64_t width, double p,
                                         uint64_t seed) {
  CircNb nb;
  nb.cnt = 0;
  // (lo, hi, other node) for right, down, left, up
  const int64_t lo[4] = {i, i, i - 1, i - width};
  const int64_t hi[4] = {i + 1, i + width, i, i};
  const bool ok[4] = {(i % width) != width - 1 && i + 1 < n, i + width < n,
                      (i % width) != 0, i - width >= 0};
  for (int d = 0; d < 4; ++d) {
    if (!ok[d]) continue;
    const uint64_t h = pair_hash(seed, lo[d], hi[d]);
    if (!(u53(h) < p)) continue;
    nb.node[nb.cnt] = lo[d] == i ? hi[d] : lo[d];
    nb.w[nb.cnt] = 0.5 + u53(mix64(h ^ kCircK));
    ++nb.cnt;
  }
  return nb;
}

__global__ void k_circ_count(int64_t n, int64_t width, double p, uint64_t seed, Scatter sc,
                             int64_t r0, int64_t r1, int32_t* counts) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = r0 + t;
  if (r >= r1) return;
  const int64_t i = scatter_inv(sc, r);
  counts[t] = 1 + circ_neighbours(i, n, width, p, seed).cnt;
}

__global__ void k_circ_fill(int64_t n, int64_t width, double p, uint64_t seed, Scatter sc,
                            int64_t r0, int64_t r1, const int64_t* __restrict__ rowptr, int nplant,
                            const double* __restrict__ plant, int32_t* col, double* val) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t r = r0 + t;
  if (r >= r1) return;
  const int64_t i = scatter_inv(sc, r);
  const CircNb nb = circ_neighbours(i, n, width, p, seed);
  double diag = 0.01;
  for (int d = 0; d < nb.cnt; ++d) diag += nb.w[d];
  const int64_t stride = nplant > 0 ? n / nplant : 0;
  if (stride > 0 && i % stride == 0 && i / stride < nplant) diag += plant[i / stride];
  int64_t c[5];
  double v[5];
  const int m = nb.cnt + 1;
  c[0] = r;
  v[0] = diag;
  for (int d = 0; d < nb.cnt; ++d) {
    c[d + 1] = scatter(sc, nb.node[d]);
    v[d + 1] = -nb.w[d];
  }
  for (int a = 1; a < m; ++a)  // insertion sort by column (<= 5 entries)
    for (int b2 = a; b2 > 0 && c[b2 - 1] > c[b2]; --b2) {
      const int64_t tc = c[b2]; c[b2] = c[b2 - 1]; c[b2 - 1] = tc;
      const double tv = v[b2]; v[b2] = v[b2 - 1]; v[b2 - 1] = tv;
    }
  const int64_t e = rowptr[t];
  for (int a = 0; a < m; ++a) {
    col[e + a] = (int32_t)c[a];
    val[e + a] = v[a];
  }
}

void circ_count(int64_t n, int64_t width, double p, uint64_t seed, int64_t r0, int64_t r1,
                int32_t* counts, hipStream_t s) {
  const int64_t m = r1 - r0;
  if (m <= 0) return;
  hipLaunchKernelGGL(k_circ_count, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, n, width,
                     p, seed, make_scatter(n, seed), r0, r1, counts);
}

void circ_fill(int64_t n, int64_t width, double p, uint64_t seed, int64_t r0, int64_t r1,
               const int64_t* rowptr, int nplant, const double* plant_dev, int32_t* col,
               double* val, hipStream_t s) {
  const int64_t m = r1 - r0;
  if (m <= 0) return;
  hipLaunchKernelGGL(k_circ_fill, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, n, width, p,
                     seed, make_scatter(n, seed), r0, r1, rowptr, nplant, plant_dev, col, val);
}

// ---- indexed halo (several ranks, unbanded A): pack the rows peers asked for, mark the
// columns a rank references outside its rows, renumber the halo tier's columns ----
__global__ void k_gather_rows(const double* __restrict__ Q, const int32_t* __restrict__ idx,
                              int64_t nrows, int b, double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nrows * b) return;
  const int64_t i = e / b;
  const int c = (int)(e - i * b);
  out[e] = Q[(int64_t)idx[i] * b + c];
}
void gather_rows(const double* Q, const int32_t* idx, int64_t nrows, int b, double* out,
                 hipStream_t s) {
  const int64_t m = nrows * b;
  if (m <= 0) return;
  hipLaunchKernelGGL(k_gather_rows, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, Q, idx,
                     nrows, b, out);
}
__global__ void k_mark_cols(const int32_t* __restrict__ col, int64_t nnz, int64_t r0, int64_t r1,
                            uint8_t* mark) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz;
       k += (int64_t)gridDim.x * blockDim.x) {
    const int64_t c = col[k];
    if (c < r0 || c >= r1) mark[c] = 1;  // idempotent byte stores: no atomics needed
  }
}
void mark_cols(const int32_t* col, int64_t nnz, int64_t r0, int64_t r1, uint8_t* mark,
               hipStream_t s) {
  if (nnz <= 0) return;
  hipLaunchKernelGGL(k_mark_cols, dim3(4096), dim3(256), 0, s, col, nnz, r0, r1, mark);
}
__global__ void k_remap_cols(int32_t* col, int64_t nnz, const int32_t* __restrict__ map) {
  for (int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nnz;
       k += (int64_t)gridDim.x * blockDim.x)
    col[k] = map[col[k]];
}
void remap_cols(int32_t* col, int64_t nnz, const int32_t* map, hipStream_t s) {
  if (nnz <= 0) return;
  hipLaunchKernelGGL(k_remap_cols, dim3(4096), dim3(256), 0, s, col, nnz, map);
}

__global__ void k_randn(double* Q, int64_t nrows, int b, int64_t r0, uint64_t seed, bool relabel,
                        Scatter perm) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nrows * b) return;
  const int64_t r = e / b;
  const int c = (int)(e - r * b);
  const int64_t id = relabel ? scatter_inv(perm, r0 + r) : r0 + r;
  const uint64_t h = mix64(seed ^ mix64((uint64_t)id * 1024u + (uint64_t)c));
  const double u1 = ((double)(h >> 11) + 0.5) * 0x1.0p-53;
  const double u2 = (double)(mix64(h) >> 11) * 0x1.0p-53;
  Q[e] = sqrt(-2.0 * log(u1)) * cospi(2.0 * u2);
}

void randn_block(double* Q, int64_t nrows, int b, int64_t r0, uint64_t seed, hipStream_t s,
                 const Scatter* perm) {
  const int64_t m = nrows * b;
  if (m <= 0) return;
  hipLaunchKernelGGL(k_randn, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, Q, nrows, b, r0,
                     seed, perm != nullptr, perm ? *perm : Scatter());
}

__global__ void k_tile_cols(int64_t nrows, const int64_t* __restrict__ rowptr,
                            const int32_t* __restrict__ col, int tile_rows, int64_t ntiles,
                            int64_t* cmin, int64_t* cmax) {
  const int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= ntiles) return;
  const int64_t ra = t * tile_rows;
  const int64_t rb = ra + tile_rows < nrows ? ra + tile_rows : nrows;
  int64_t mn = INT64_MAX, mx = -1;
  for (int64_t r = ra; r < rb; ++r) {
    const int64_t s = rowptr[r], e = rowptr[r + 1];
    if (e > s) {  // columns are sorted within a row
      mn = col[s] < mn ? col[s] : mn;
      mx = col[e - 1] > mx ? col[e - 1] : mx;
    }
  }
  cmin[t] = mx < 0 ? 0 : mn;
  cmax[t] = mx;
}

void tile_col_range(const CsrDev& A, int tile_rows, int64_t* cmin, int64_t* cmax, hipStream_t s) {
  const int64_t nt = (A.nrows + tile_rows - 1) / tile_rows;
  if (nt <= 0) return;
  hipLaunchKernelGGL(k_tile_cols, dim3((unsigned)((nt + 255) / 256)), dim3(256), 0, s, A.nrows,
                     A.rowptr, A.col, tile_rows, nt, cmin, cmax);
}

__global__ void k_c2r(const double* __restrict__ src, int64_t nrows, int w, double* __restrict__ dst) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // e = c*nrows + r
  if (e >= nrows * w) return;
  const int64_t c = e / nrows, r = e - c * nrows;
  dst[r * w + c] = src[e];
}
__global__ void k_r2c(const double* __restrict__ src, int64_t nrows, int w, double* __restrict__ dst) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;  // e = c*nrows + r
  if (e >= nrows * w) return;
  const int64_t c = e / nrows, r = e - c * nrows;
  dst[e] = src[r * w + c];
}
// The same transposes through LDS for w <= 64: a workgroup moves 64 rows, reading the row-major
// side as one contiguous run and each column's 64 values as one, where the element-wise kernels
// above read (or write) with a w-element stride — at n = 1e7, w = 20 (the Ritz vectors) the
// strided side touched every 128-B line once per column it holds (~4 ms instead of ~0.6)
template <bool R2C>
__global__ __launch_bounds__(256) void k_transpose64(const double* __restrict__ src, int64_t nrows, int w,
                                                     double* __restrict__ dst) {
  __shared__ double t[64][65];
  const int64_t r0 = (int64_t)blockIdx.x * 64;
  const int rows = nrows - r0 < 64 ? (int)(nrows - r0) : 64;
  const int m = rows * w;
  for (int idx = threadIdx.x; idx < m; idx += 256) {
    if (R2C) {  // row-major run [r0 w, (r0 + rows) w)
      t[idx / w][idx % w] = src[r0 * w + idx];
    } else {    // column c, rows r0 .. r0 + rows
      const int c = idx / rows, r = idx - c * rows;
      t[r][c] = src[(int64_t)c * nrows + r0 + r];
    }
  }
  __syncthreads();
  for (int idx = threadIdx.x; idx < m; idx += 256) {
    if (R2C) {
      const int c = idx / rows, r = idx - c * rows;
      dst[(int64_t)c * nrows + r0 + r] = t[r][c];
    } else {
      dst[r0 * w + idx] = t[idx / w][idx % w];
    }
  }
}
void colmajor_to_rowmajor(const double* src, int64_t nrows, int w, double* dst, hipStream_t s) {
  const int64_t m = nrows * w;
  if (m <= 0) return;
  if (w <= 64) {
    hipLaunchKernelGGL(k_transpose64<false>, dim3((unsigned)((nrows + 63) / 64)), dim3(256), 0, s, src, nrows,
                       w, dst);
    return;
  }
  hipLaunchKernelGGL(k_c2r, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, src, nrows, w, dst);
}
void rowmajor_to_colmajor(const double* src, int64_t nrows, int w, double* dst, hipStream_t s) {
  const int64_t m = nrows * w;
  if (m <= 0) return;
  if (w <= 64) {
    hipLaunchKernelGGL(k_transpose64<true>, dim3((unsigned)((nrows + 63) / 64)), dim3(256), 0, s, src, nrows,
                       w, dst);
    return;
  }
  hipLaunchKernelGGL(k_r2c, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, src, nrows, w, dst);
}

}  // namespace rbl
