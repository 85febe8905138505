// tsmm.hip — tall-skinny fp64 MFMA kernels for gfx950.
//
// These replace every cuBLAS gemm of the reference's block step:
//   * Gram  C = W^T X   — A_i = Q_i^T U (RBL_gpu.jl:153,178), local-reorth coefficient
//     (RBL_gpu.jl:87), partial-reorth coefficients against the Krylov basis
//     (RBL_gpu.jl:33,39,50,52) and the CholQR Gram matrices that replace cuSOLVER geqrf.
//   * update Y = beta Y + alpha X C — U -= Q_i A_i (:154,179), local / partial reorth
//     updates (:88, :34,40,51,53), CholQR apply, and the Ritz projection (:121).
//
// Both are v_mfma_f64_16x16x4f64 tiles (one f64 per lane for A and B; C/D: col = lane&15,
// row = (lane>>4) + 4*reg).  Memory layout: every n x w panel is row-major, so a 16-lane
// quad reads 128 contiguous bytes.  Gram partials go to a slab [split][a][c] reduced in a
// fixed order by reduce_slab (bitwise reproducible, no atomics).
#include <cstdlib>

#include <algorithm>

#include "kernels.hpp"

namespace rbl {

typedef double d4 __attribute__((ext_vector_type(4)));

__device__ inline d4 mfma16(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}

// ----------------------------------------------------------------------------------------
// Gram partials
// ----------------------------------------------------------------------------------------
template <int AT, int CT>
__global__ __launch_bounds__(256) void k_gram(int64_t nrows, PanelRun W, Panels X, double* slab,
                                              int splits, int ncg, int nag, int64_t rows_per,
                                              const int* skip) {
  if (skip && *skip) return;
  const int lane = threadIdx.x & 63;
  const int wid = blockIdx.x * 4 + (threadIdx.x >> 6);
  // job = (panel j, W column group ag of 16 AT columns, X column group cg of 16 CT columns)
  const int njobs = W.count * nag * ncg;
  const int job = wid % njobs;
  const int s = wid / njobs;
  if (s >= splits) return;
  const int j = job % W.count;
  const int ag = (job / W.count) % nag;
  const int cg = job / (W.count * nag);
  const int w = W.w, xw = X.w;
  const int KC = X.count * xw;
  const int KW = W.count * w;
  const int li = lane & 15, q = lane >> 4;

  const int64_t r_begin = (int64_t)s * rows_per;
  const int64_t r_end = r_begin + rows_per < nrows ? r_begin + rows_per : nrows;

  const double* wp[AT];
  bool wv[AT];
#pragma unroll
  for (int at = 0; at < AT; ++at) {
    const int a = (ag * AT + at) * 16 + li;
    wv[at] = a < w;
    wp[at] = W.base + (int64_t)j * W.stride + (wv[at] ? a : 0);
  }
  const double* xp[CT];
  bool xv[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int c = (cg * CT + ct) * 16 + li;
    xv[ct] = c < KC;
    const int t = xv[ct] ? c / xw : 0;
    xp[ct] = X.ptr[t] + (xv[ct] ? c - t * xw : 0);
  }
  d4 acc[AT][CT];
#pragma unroll
  for (int at = 0; at < AT; ++at)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[at][ct] = d4{0.0, 0.0, 0.0, 0.0};

  // main loop: 4 rows per MFMA k-step, lane quad q owns row r0 + q
  int64_t r0 = r_begin;
  for (; r0 + 4 <= r_end; r0 += 4) {
    const int64_t row = r0 + q;
    double av[AT], xv_[CT];
#pragma unroll
    for (int at = 0; at < AT; ++at) av[at] = wv[at] ? wp[at][row * w] : 0.0;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) xv_[ct] = xv[ct] ? xp[ct][row * xw] : 0.0;
#pragma unroll
    for (int at = 0; at < AT; ++at)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[at][ct] = mfma16(av[at], xv_[ct], acc[at][ct]);
  }
  if (r0 < r_end) {  // ragged tail (wave-uniform branch)
    const int64_t row = r0 + q;
    const bool rv = row < r_end;
    double av[AT], xv_[CT];
#pragma unroll
    for (int at = 0; at < AT; ++at) av[at] = (rv && wv[at]) ? wp[at][row * w] : 0.0;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) xv_[ct] = (rv && xv[ct]) ? xp[ct][row * xw] : 0.0;
#pragma unroll
    for (int at = 0; at < AT; ++at)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[at][ct] = mfma16(av[at], xv_[ct], acc[at][ct]);
  }

  double* out = slab + (int64_t)s * KW * KC;
#pragma unroll
  for (int at = 0; at < AT; ++at)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int a = (ag * AT + at) * 16 + q + 4 * reg;
        const int c = (cg * CT + ct) * 16 + li;
        if (a < w && c < KC) out[(int64_t)(j * w + a) * KC + c] = acc[at][ct][reg];
      }
}

static int tiles16(int x) { return (x + 15) / 16; }
static int pick_at(int w) { int t = tiles16(w); return t <= 1 ? 1 : (t <= 2 ? 2 : 4); }

int gram_splits(int64_t nrows, int nW, int w, int xcols) {
  if (xcols % w == 0 && gram44_ok(nrows, nW, w, xcols / w, w)) return gram44_splits(nrows, nW, w);
  const int ctt = tiles16(xcols);
  const int ct = ctt <= 1 ? 1 : (ctt <= 2 ? 2 : 4);
  const int ncg = (ctt + ct - 1) / ct;
  const int64_t njobs = (int64_t)nW * ((tiles16(w) + pick_at(w) - 1) / pick_at(w)) * ncg;
  int64_t splits = (4096 + njobs - 1) / njobs;
  const int64_t max_by_rows = (nrows + 63) / 64;
  if (splits > max_by_rows) splits = max_by_rows;
  // keep the slab <= 256 MB
  const int64_t per = (int64_t)nW * w * xcols * 8;
  const int64_t max_by_mem = per > 0 ? (256ll << 20) / per : splits;
  if (splits > max_by_mem) splits = max_by_mem;
  if (splits < 1) splits = 1;
  return (int)splits;
}

template <int AT, int CT>
static void launch_gram_t(int64_t nrows, const PanelRun& W, const Panels& X, double* slab,
                          int splits, int ncg, const int* skip, hipStream_t s) {
  int64_t rows_per = (nrows + splits - 1) / splits;
  rows_per = (rows_per + 3) / 4 * 4;
  const int nag = (tiles16(W.w) + AT - 1) / AT;  // W wider than 16 AT columns (b > 64)
  const int64_t waves = (int64_t)W.count * nag * ncg * splits;
  const int blocks = (int)((waves + 3) / 4);
  hipLaunchKernelGGL((k_gram<AT, CT>), dim3(blocks), dim3(256), 0, s, nrows, W, X, slab, splits,
                     ncg, nag, rows_per, skip);
}

void gram_partial(int64_t nrows, const PanelRun& W, const Panels& X, double* slab, int splits,
                  const int* skip, hipStream_t s) {
  if (gram44_ok(nrows, W.count, W.w, X.count, X.w)) return gram44_partial(nrows, W, X, slab, splits, skip, s);
  const int at = pick_at(W.w);
  const int ctt = tiles16(X.count * X.w);
  const int ct = ctt <= 1 ? 1 : (ctt <= 2 ? 2 : 4);
  const int ncg = (ctt + ct - 1) / ct;
#define RBL_GRAM_CASE(A_, C_) \
  if (at == A_ && ct == C_) return launch_gram_t<A_, C_>(nrows, W, X, slab, splits, ncg, skip, s);
  RBL_GRAM_CASE(1, 1) RBL_GRAM_CASE(1, 2) RBL_GRAM_CASE(1, 4)
  RBL_GRAM_CASE(2, 1) RBL_GRAM_CASE(2, 2) RBL_GRAM_CASE(2, 4)
  RBL_GRAM_CASE(4, 1) RBL_GRAM_CASE(4, 2) RBL_GRAM_CASE(4, 4)
#undef RBL_GRAM_CASE
}

// ----------------------------------------------------------------------------------------
// Deterministic slab reduction
// ----------------------------------------------------------------------------------------
// 256 threads = 16 elements x 16 split lanes; split lane j sums splits j, j+16, ... (4
// independent chains to keep loads in flight), then a fixed LDS tree over the 16 lanes.
__global__ __launch_bounds__(256) void k_reduce(const double* __restrict__ slab, int splits,
                                                int64_t len, double* __restrict__ out,
                                                const int* skip) {
  if (skip && *skip) return;
  __shared__ double part[16][17];
  const int el = threadIdx.x & 15, j = threadIdx.x >> 4;
  const int64_t e = (int64_t)blockIdx.x * 16 + el;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (e < len) {
    int s = j;
    // unrolled: up to 16 loads in flight per lane (the sums keep their order: same bits)
#pragma unroll 4
    for (; s + 48 < splits; s += 64) {
      a0 += slab[(int64_t)s * len + e];
      a1 += slab[(int64_t)(s + 16) * len + e];
      a2 += slab[(int64_t)(s + 32) * len + e];
      a3 += slab[(int64_t)(s + 48) * len + e];
    }
    for (; s < splits; s += 16) a0 += slab[(int64_t)s * len + e];
  }
  part[j][el] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  if (j == 0 && e < len) {
    double acc = 0.0;
#pragma unroll
    for (int t = 0; t < 16; ++t) acc += part[t][el];
    out[e] = acc;
  }
}

// Many splits (the partial-reorth update's local-reorth Gram: one partial per 128-row tile,
// ~78 k at C4a): sum fixed chunks of splits in parallel (red_chunk per chunk) until at most
// 64 remain, each level into the scratch after the previous one, then k_reduce — a fixed order
// (bitwise reproducible); one k_reduce pass over 78 k partials is latency-bound (16 split lanes
// per element, 64 workgroups): 310 us against ~130 us.
// Chunk 32 (round 5): the first level's grid is then ~splits / 32 x len / 256 workgroups whose
// threads sum 32 partials each (8 rounds of 4 loads) — at n = 1.25e6 (9,766 partials) 1,224
// workgroups instead of 156 that summed 256 each (64 dependent rounds, 40 us).  RBL_RED_CHUNK=0:
// the earlier rule (256 above 4,096 partials, else 16), for A/B.
#ifdef RBL_VARIANTS
static int red_chunk(int splits) {
  const char* e = std::getenv("RBL_RED_CHUNK");  // read per call: the slab is sized by
  const int mode = e ? std::atoi(e) : 32;          // rbl_start under the same setting
  if (mode <= 0) return splits > 4096 ? 256 : 16;
  return std::max(2, mode);                        // (1 would never shrink the level)
}
#else
static constexpr int red_chunk(int) { return 32; }
#endif
int reduce_scratch_splits(int splits) {
  int tot = 0;
  while (splits > 64) {
    splits = (splits + red_chunk(splits) - 1) / red_chunk(splits);
    tot += splits;
  }
  return tot;
}
__global__ __launch_bounds__(256) void k_reduce_chunks(const double* __restrict__ slab, int splits,
                                                       int chunk, int64_t len,
                                                       double* __restrict__ part) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int c = blockIdx.y;
  if (e >= len) return;
  const int s0 = c * chunk, s1 = s0 + chunk < splits ? s0 + chunk : splits;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  int sp = s0;
  for (; sp + 3 < s1; sp += 4) {
    a0 += slab[(int64_t)sp * len + e];
    a1 += slab[(int64_t)(sp + 1) * len + e];
    a2 += slab[(int64_t)(sp + 2) * len + e];
    a3 += slab[(int64_t)(sp + 3) * len + e];
  }
  for (; sp < s1; ++sp) a0 += slab[(int64_t)sp * len + e];
  part[(int64_t)c * len + e] = (a0 + a1) + (a2 + a3);
}

// The b x b Grams of a block step (len = b^2 <= 4096, one partial per row-op workgroup: ~500
// at n = 1.25e6): 4 elements x 64 split lanes per workgroup, so len / 4 workgroups cover the
// chip and a lane's sums are 2 rounds of 4 independent loads instead of k_reduce's 8 (a latency
// kernel between two dependent launches, ~5 per step); then a fixed LDS tree over the 64 lanes.
__global__ __launch_bounds__(256) void k_reduce_wide(const double* __restrict__ slab, int splits,
                                                     int64_t len, double* __restrict__ out,
                                                     const int* skip) {
  if (skip && *skip) return;
  __shared__ double part[64][5];
  const int el = threadIdx.x & 3, j = threadIdx.x >> 2;
  const int64_t e = (int64_t)blockIdx.x * 4 + el;
  double a0 = 0.0, a1 = 0.0, a2 = 0.0, a3 = 0.0;
  if (e < len) {
    int s = j;
#pragma unroll 2
    for (; s + 192 < splits; s += 256) {
      a0 += slab[(int64_t)s * len + e];
      a1 += slab[(int64_t)(s + 64) * len + e];
      a2 += slab[(int64_t)(s + 128) * len + e];
      a3 += slab[(int64_t)(s + 192) * len + e];
    }
    for (; s < splits; s += 64) a0 += slab[(int64_t)s * len + e];
  }
  part[j][el] = (a0 + a1) + (a2 + a3);
  __syncthreads();
  // 64 -> 1 in a fixed pairwise order: lane pairs (t, t + w) for w = 32, 16, ..., 1
  for (int w = 32; w >= 1; w >>= 1) {
    if (j < w) part[j][el] += part[j + w][el];
    __syncthreads();
  }
  if (j == 0 && e < len) out[e] = part[0][el];
}

void reduce_slab(const double* slab, int splits, int64_t len, double* out, const int* skip,
                 hipStream_t s) {
#ifdef RBL_VARIANTS
  const bool narrow = std::getenv("RBL_REDUCE_NARROW") != nullptr;  // k_reduce for every len (A/B)
#else
  constexpr bool narrow = false;
#endif
  if (len <= 4096 && splits > 64 && !narrow) {
    hipLaunchKernelGGL(k_reduce_wide, dim3((unsigned)((len + 3) / 4)), dim3(256), 0, s, slab, splits, len,
                       out, skip);
    return;
  }
  const int blocks = (int)((len + 15) / 16);
  hipLaunchKernelGGL(k_reduce, dim3(blocks), dim3(256), 0, s, slab, splits, len, out, skip);
}

void reduce_slab_many(double* slab, int splits, int64_t len, double* out, hipStream_t s) {
  while (splits > 64) {  // scratch: reduce_scratch_splits(splits) x len after the partials
    const int chunk = red_chunk(splits), nc = (splits + chunk - 1) / chunk;
    double* part = slab + (int64_t)splits * len;
    hipLaunchKernelGGL(k_reduce_chunks, dim3((unsigned)((len + 255) / 256), (unsigned)nc), dim3(256), 0,
                       s, slab, splits, chunk, len, part);
    slab = part;
    splits = nc;
  }
  reduce_slab(slab, splits, len, out, nullptr, s);
}

// ----------------------------------------------------------------------------------------
// Y = beta*Y + alpha * X * C
// ----------------------------------------------------------------------------------------
template <int RT, int CT>
__global__ __launch_bounds__(256) void k_tsmm(int64_t nrows, PanelRun X, const double* __restrict__ C,
                                              int ldc, Panels Y, double alpha, double beta,
                                              int ncg, const int* skip) {
  if (skip && *skip) return;
  const int lane = threadIdx.x & 63;
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int cg = (int)(wid % ncg);
  const int64_t rg = wid / ncg;
  const int64_t rowbase = rg * (16 * RT);
  if (rowbase >= nrows) return;
  const int li = lane & 15, q = lane >> 4;
  const int xw = X.w;
  const int K = X.count * xw;
  const int KY = Y.count * Y.w;

  bool rv[RT];
  int64_t arow[RT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt) {
    arow[rt] = rowbase + rt * 16 + li;
    rv[rt] = arow[rt] < nrows;
  }
  int cc[CT];
  bool cv[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    cc[ct] = (cg * CT + ct) * 16 + li;
    cv[ct] = cc[ct] < KY;
  }
  d4 acc[RT][CT];
#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = d4{0.0, 0.0, 0.0, 0.0};

  // k = panel*xw + col; lane quad q owns k = k0 + q
  int panel = 0, col = q;          // running (panel, col) of k = k0 + q
  while (col >= xw && panel < X.count) { col -= xw; ++panel; }
  for (int k0 = 0; k0 < K; k0 += 4) {
    const int k = k0 + q;
    const bool kv = k < K;
    const double* xpan = X.base + (int64_t)panel * X.stride;
    double a[RT], bb[CT];
#pragma unroll
    for (int rt = 0; rt < RT; ++rt) a[rt] = (kv && rv[rt]) ? xpan[arow[rt] * xw + col] : 0.0;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) bb[ct] = (kv && cv[ct]) ? C[(int64_t)k * ldc + cc[ct]] : 0.0;
#pragma unroll
    for (int rt = 0; rt < RT; ++rt)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) acc[rt][ct] = mfma16(a[rt], bb[ct], acc[rt][ct]);
    col += 4;
    while (col >= xw) { col -= xw; ++panel; }
  }

#pragma unroll
  for (int rt = 0; rt < RT; ++rt)
#pragma unroll
    for (int ct = 0; ct < CT; ++ct)
#pragma unroll
      for (int reg = 0; reg < 4; ++reg) {
        const int64_t r = rowbase + rt * 16 + q + 4 * reg;
        const int c = (cg * CT + ct) * 16 + li;
        if (r < nrows && c < KY) {
          const int t = c / Y.w;
          double* yp = const_cast<double*>(Y.ptr[t]) + r * Y.w + (c - t * Y.w);
          const double v = alpha * acc[rt][ct][reg];
          *yp = beta == 0.0 ? v : beta * (*yp) + v;
        }
      }
}

template <int RT, int CT>
static void launch_tsmm_t(int64_t nrows, const PanelRun& X, const double* C, int ldc,
                          const Panels& Y, double alpha, double beta, int ncg, const int* skip,
                          hipStream_t s) {
  const int64_t rgs = (nrows + 16 * RT - 1) / (16 * RT);
  const int64_t waves = rgs * ncg;
  const int64_t blocks = (waves + 3) / 4;
  hipLaunchKernelGGL((k_tsmm<RT, CT>), dim3((unsigned)blocks), dim3(256), 0, s, nrows, X, C, ldc,
                     Y, alpha, beta, ncg, skip);
}

void tsmm(int64_t nrows, const PanelRun& X, const double* C, int ldc, const Panels& Y,
          double alpha, double beta, const int* skip, hipStream_t s, double* xslab, int* xgrid) {
  if (xgrid) *xgrid = 0;
  if (tsmm44_ok(X.w, Y.count * Y.w, Y.w))
    return tsmm44(nrows, X, C, ldc, Y, alpha, beta, skip, s, xslab, xgrid);
  const int ctt = tiles16(Y.count * Y.w);
  const int ct = ctt <= 1 ? 1 : (ctt <= 2 ? 2 : 4);
  const int ncg = (ctt + ct - 1) / ct;
  // in-place use (Y aliasing X) is race-free only when one wave owns whole rows (ncg == 1,
  // i.e. Y.count*Y.w <= 64); the API layer only aliases for the b x b CholQR apply.
  if (ct == 1) return launch_tsmm_t<2, 1>(nrows, X, C, ldc, Y, alpha, beta, ncg, skip, s);
  if (ct == 2) return launch_tsmm_t<2, 2>(nrows, X, C, ldc, Y, alpha, beta, ncg, skip, s);
  return launch_tsmm_t<2, 4>(nrows, X, C, ldc, Y, alpha, beta, ncg, skip, s);
}

}  // namespace rbl
