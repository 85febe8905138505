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

__global__ void k_randn(double* Q, int64_t nrows, int b, int64_t r0, uint64_t seed) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nrows * b) return;
  const int64_t r = e / b;
  const int c = (int)(e - r * b);
  const uint64_t h = mix64(seed ^ mix64((uint64_t)(r0 + r) * 1024u + (uint64_t)c));
  const double u1 = ((double)(h >> 11) + 0.5) * 0x1.0p-53;
  const double u2 = (double)(mix64(h) >> 11) * 0x1.0p-53;
  Q[e] = sqrt(-2.0 * log(u1)) * cospi(2.0 * u2);
}

void randn_block(double* Q, int64_t nrows, int b, int64_t r0, uint64_t seed, hipStream_t s) {
  const int64_t m = nrows * b;
  if (m <= 0) return;
  hipLaunchKernelGGL(k_randn, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, Q, nrows, b, r0,
                     seed);
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
void colmajor_to_rowmajor(const double* src, int64_t nrows, int w, double* dst, hipStream_t s) {
  const int64_t m = nrows * w;
  if (m <= 0) return;
  hipLaunchKernelGGL(k_c2r, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, src, nrows, w, dst);
}
void rowmajor_to_colmajor(const double* src, int64_t nrows, int w, double* dst, hipStream_t s) {
  const int64_t m = nrows * w;
  if (m <= 0) return;
  hipLaunchKernelGGL(k_r2c, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, src, nrows, w, dst);
}

}  // namespace rbl
