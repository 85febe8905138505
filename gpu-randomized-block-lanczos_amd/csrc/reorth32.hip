// reorth32.hip — the fp32 Krylov basis (mixed-precision mode, RBL_gpu.jl with
// FLOAT = Float32: SURVEY P9): partial and local reorthogonalisation on fp32 blocks with
// v_mfma_f32_16x16x4_f32 (exact f32 fma chains, 64 FLOP/clk/SIMD = 2x the fp64 MFMA rate,
// half the bytes per basis element), and the fp32 <-> fp64 conversions between the basis and
// the fp64 SpMM / 3-term / QR path (RBL_gpu.jl:172-174, 180-182: copyto! between Qg and Qg_d).
//
// v_mfma_f32_16x16x4_f32 (cdna_hip_programming.md 'FP32-input MFMA'): lane l holds
//   A[i = l&15][k = l>>4], B[k = l>>4][j = l&15], D[row 4 (l>>4) + v][col l&15], v = reg 0..3.
#include <cstdlib>

#include "kernels.hpp"

namespace rbl {

typedef float f4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ f4v mfma16(float a, float b, f4v c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// ----------------------------------------------------------------------------------------
// Gram C = W^T X (fp32 in, fp32 MFMA accumulation per split; splits summed in fp64 by
// reduce_slab): one Krylov panel per wave, 4 waves per workgroup, X rows staged in LDS in
// 16-row chunks.  X chunk image: column c of row r at r * 64 + 4 (c & 15) + (c >> 4), so one
// ds_read_b128 hands a lane its B operand for all four 16-column tiles.
// ----------------------------------------------------------------------------------------
constexpr int kG32Waves = 4;
// rows per X chunk (one barrier per chunk): 16 or 32
#ifndef RBL_G32_ROWS
#define RBL_G32_ROWS 32
#endif
constexpr int kG32Rows = RBL_G32_ROWS;
// basis operand prefetch depth in chunks (1 or 2)
#ifndef RBL_G32_PF
#define RBL_G32_PF 1
#endif
static_assert((kG32Rows == 16 || kG32Rows == 32) && kG32Rows <= kRowPad32, "fp32 Gram chunk rows");

template <int W, int NX>
__global__ __launch_bounds__(256) void k_gram32(int64_t nrows, const float* __restrict__ Wb,
                                                int64_t wstride, int nW, const float* __restrict__ X0,
                                                const float* __restrict__ X1, double* __restrict__ slab,
                                                int npg, int64_t rows_per) {
  constexpr int KC = NX * W;        // X columns
  constexpr int CT = KC / 16;       // 16-column tiles of X (1..4)
  constexpr int AT = W / 16;        // 16-column tiles of the panel (1..2)
  constexpr int KS = kG32Rows / 4;  // k steps (4 rows each) per chunk
  constexpr int XR = kG32Rows / 16; // X rows staged per thread per chunk
  __shared__ __attribute__((aligned(16))) float xs[2][kG32Rows * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, c16 = lane & 15;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, t = bid >> 3;  // XCD-aware: a split's panel groups share an L2
  const int pg = t % npg;
  const int64_t s = (int64_t)(t / npg) * 8 + xcd;
  const int64_t r_begin = s * rows_per;
  const int64_t r_end = r_begin + rows_per < nrows ? r_begin + rows_per : nrows;
  const int j = pg * kG32Waves + wave;
  const bool active = j < nW;
  const float* wp = Wb + (int64_t)(active ? j : 0) * wstride + c16;

  f4v acc[AT][CT];
#pragma unroll
  for (int a = 0; a < AT; ++a)
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[a][c] = f4v{0.f, 0.f, 0.f, 0.f};

  // X staging: thread (row = tid / 16, cc = tid % 16) moves X[row][cc + 16 ct] (ct < CT).
  // A partial last chunk is shifted back to end at r_end (wave-uniform row base, no per-lane
  // clamps) and its rows below rc0 — already counted — zeroed on the X side, as in
  // reorth.hip's k_gram44.  With nrows < kG32Rows the chunk starts at row 0 and over-reads into
  // the next basis slot or the zeroed allocation pad (kRowPad32, rbl_start): finite rows met
  // by zero X.
  const int xrow = tid >> 4, xcc = tid & 15;
  const float* xsl[CT];
#pragma unroll
  for (int ct = 0; ct < CT; ++ct) {
    const int c = xcc + 16 * ct;
    xsl[ct] = ((NX == 2 && c >= W) ? X1 + (c - W) : X0 + c) + (int64_t)xrow * W;
  }
  const float* wl = wp + q * W;
  auto shift = [&](int64_t rc0) -> int64_t {
    const int64_t r = rc0 < r_end - kG32Rows ? rc0 : r_end - kG32Rows;
    return r > 0 ? r : 0;
  };
  auto load_x = [&](int64_t rc0, float (&xr)[XR][CT]) {
    const int64_t o = shift(rc0) * W;
#pragma unroll
    for (int h = 0; h < XR; ++h)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) xr[h][ct] = xsl[ct][o + 16 * h * W];
  };
  auto store_x = [&](int buf, int64_t rc0, const float (&xr)[XR][CT]) {
#pragma unroll
    for (int h = 0; h < XR; ++h) {
      const int64_t row = shift(rc0) + xrow + 16 * h;
      const bool ok = row >= rc0 && row < r_end;
      float* d = &xs[buf][(xrow + 16 * h) * 64 + 4 * xcc];
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) d[ct] = ok ? xr[h][ct] : 0.f;
    }
  };
  auto load_a = [&](int64_t rc0, float (&ar)[KS][AT]) {
    const float* p = wl + shift(rc0) * W;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int a = 0; a < AT; ++a) ar[ks][a] = p[4 * ks * W + 16 * a];
  };

  const int64_t nchunks = r_end > r_begin ? (r_end - r_begin + kG32Rows - 1) / kG32Rows : 0;
  float xr[XR][CT];
  auto mma = [&](int64_t ch, const float (&acur)[KS][AT]) {
    const float* xb = xs[ch & 1] + 4 * c16;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const f4v bv = *reinterpret_cast<const f4v*>(xb + (4 * ks + q) * 64);
#pragma unroll
      for (int a = 0; a < AT; ++a)
#pragma unroll
        for (int c = 0; c < CT; ++c) acc[a][c] = mfma16(acur[ks][a], bv[c], acc[a][c]);
    }
  };
#if RBL_G32_PF >= 2
  // basis operands two chunks ahead in three rotating register sets (as k_gram44)
  float a0[KS][AT], a1[KS][AT], a2[KS][AT];
  if (nchunks > 0) {
    load_x(r_begin, xr);
    store_x(0, r_begin, xr);
    load_a(r_begin, a0);
    load_a(r_begin + kG32Rows, a1);
  }
  __syncthreads();
  auto step = [&](int64_t ch, const float (&acur)[KS][AT], float (&afut)[KS][AT]) {
    const int64_t rc0 = r_begin + ch * kG32Rows;
    load_x(rc0 + kG32Rows, xr);
    load_a(rc0 + 2 * kG32Rows, afut);
    if (active && ch < nchunks) mma(ch, acur);  // no loads inside
    store_x((int)((ch + 1) & 1), rc0 + kG32Rows, xr);
    __syncthreads();
  };
  for (int64_t ch = 0; ch < nchunks; ch += 3) {
    step(ch, a0, a2);
    step(ch + 1, a1, a0);
    step(ch + 2, a2, a1);
  }
#else
  float acur[KS][AT], anext[KS][AT];
  if (nchunks > 0) {
    load_x(r_begin, xr);
    store_x(0, r_begin, xr);
    load_a(r_begin, acur);
  }
  __syncthreads();
  for (int64_t ch = 0; ch < nchunks; ++ch) {
    const int64_t rc0 = r_begin + ch * kG32Rows;
    load_x(rc0 + kG32Rows, xr);  // unconditional (clamped): see reorth.hip
    load_a(rc0 + kG32Rows, anext);
    if (active) mma(ch, acur);
    store_x((int)((ch + 1) & 1), rc0 + kG32Rows, xr);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int a = 0; a < AT; ++a) acur[ks][a] = anext[ks][a];
    __syncthreads();
  }
#endif
  if (!active) return;
  // D[a][c] tile (16 x 16): lane holds rows 4q + v, column c16 of the tile
  double* out = slab + (s * (int64_t)nW * W + (int64_t)j * W) * KC;
#pragma unroll
  for (int a = 0; a < AT; ++a)
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
      for (int v = 0; v < 4; ++v)
        out[(int64_t)(16 * a + 4 * q + v) * KC + 16 * c + c16] = (double)acc[a][c][v];
}

// The same Gram on v_mfma_f32_32x32x2f32 (b = 32, X = [Q_i, Q_{i-1}]): one 32 x 32 output tile
// per X panel, 4096 flops per instruction (the shape measured 149 vs 136 TF/s for 16x16x4 in a
// register loop, tools/mfma_probe.hip).  Step s of a chunk takes rows 2s and 2s + 1: lane l
// holds A[i = l % 32][k = l / 32] = W[2s + l / 32][l % 32], i.e. one contiguous 256-B load of
// the two rows per step, and B[k][j] = X[2s + k][j] (+32 for the second panel), adjacent in the
// LDS image (row r, column c at r * 64 + 2 (c % 32) + c / 32) so one ds_read_b64 per step feeds
// both tiles.  D[i][j]: lane l, register v holds i = 4 (l / 32) + (v % 4) + 8 (v / 4), j = l % 32.
#ifndef RBL_G32_MFMA32
#define RBL_G32_MFMA32 1
#endif
typedef float f16v __attribute__((ext_vector_type(16)));
__global__ __launch_bounds__(256) void k_gram32x(int64_t nrows, const float* __restrict__ Wb,
                                                 int64_t wstride, int nW, const float* __restrict__ X0,
                                                 const float* __restrict__ X1, double* __restrict__ slab,
                                                 int npg, int64_t rows_per) {
  constexpr int W = 32, KC = 64, NS = kG32Rows / 2;  // k steps (2 rows each) per chunk
  constexpr int XE = kG32Rows * KC / 256;            // X elements staged per thread per chunk
  __shared__ __attribute__((aligned(16))) float xs[2][kG32Rows * KC];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int bid = blockIdx.x;
  const int xcd = bid & 7, t = bid >> 3;  // XCD-aware: a split's panel groups share an L2
  const int pg = t % npg;
  const int64_t s = (int64_t)(t / npg) * 8 + xcd;
  const int64_t r_begin = s * rows_per;
  const int64_t r_end = r_begin + rows_per < nrows ? r_begin + rows_per : nrows;
  const int j = pg * kG32Waves + wave;
  const bool active = j < nW;
  const float* wpan = Wb + (int64_t)(active ? j : 0) * wstride;  // wave-uniform

  f16v acc[2];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[tt][v] = 0.f;

  auto shift = [&](int64_t rc0) -> int64_t {
    const int64_t r = rc0 < r_end - kG32Rows ? rc0 : r_end - kG32Rows;
    return r > 0 ? r : 0;
  };
  // X staging: thread (row = e / 64, column c = e % 64) for e = 4 tid + 1024 h .. + 3 (float4 of
  // one panel: 4 consecutive columns of the same panel)
  auto load_x = [&](int64_t rc0, f4v (&xr)[XE / 4]) {
    const int64_t rb = shift(rc0);
#pragma unroll
    for (int h = 0; h < XE / 4; ++h) {
      const int e = 4 * tid + 1024 * h, row = e / KC, c = e % KC;
      const float* src = (c < W ? X0 + c : X1 + (c - W)) + (rb + row) * W;
      xr[h] = *reinterpret_cast<const f4v*>(src);
    }
  };
  auto store_x = [&](int buf, int64_t rc0, const f4v (&xr)[XE / 4]) {
    const int64_t rb = shift(rc0);
#pragma unroll
    for (int h = 0; h < XE / 4; ++h) {
      const int e = 4 * tid + 1024 * h, row = e / KC, c = e % KC;
      const bool ok = rb + row >= rc0 && rb + row < r_end;
      float* d = &xs[buf][row * KC + 2 * (c % W) + c / W];
#pragma unroll
      for (int u = 0; u < 4; ++u) d[2 * u] = ok ? xr[h][u] : 0.f;
    }
  };
  auto load_a = [&](int64_t rc0, float (&ar)[NS]) {
    const float* p = wpan + shift(rc0) * W;  // uniform
#pragma unroll
    for (int st = 0; st < NS; ++st) ar[st] = p[(unsigned)(2 * st * W + lane)];
  };

  const int64_t nchunks = r_end > r_begin ? (r_end - r_begin + kG32Rows - 1) / kG32Rows : 0;
  f4v xr[XE / 4];
  float acur[NS], anext[NS];
  if (nchunks > 0) {
    load_x(r_begin, xr);
    store_x(0, r_begin, xr);
    load_a(r_begin, acur);
  }
  __syncthreads();
  for (int64_t ch = 0; ch < nchunks; ++ch) {
    const int64_t rc0 = r_begin + ch * kG32Rows;
    load_x(rc0 + kG32Rows, xr);  // unconditional (clamped): see reorth.hip
    load_a(rc0 + kG32Rows, anext);
    if (active) {
      const float* xb = xs[ch & 1] + 2 * lane;
#pragma unroll
      for (int st = 0; st < NS; ++st) {
        const float2 bv = *reinterpret_cast<const float2*>(xb + st * 2 * KC);
        acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(acur[st], bv.x, acc[0], 0, 0, 0);
        acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(acur[st], bv.y, acc[1], 0, 0, 0);
      }
    }
    store_x((int)((ch + 1) & 1), rc0 + kG32Rows, xr);
#pragma unroll
    for (int st = 0; st < NS; ++st) acur[st] = anext[st];
    __syncthreads();
  }
  if (!active) return;
  double* out = slab + (s * (int64_t)nW * W + (int64_t)j * W) * KC;
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int v = 0; v < 16; ++v) {
      const int a = 4 * (lane / 32) + (v % 4) + 8 * (v / 4);
      out[(int64_t)a * KC + W * tt + (lane % 32)] = (double)acc[tt][v];
    }
}

// The local-reorth Gram C = Q_{i-1}^T Q_i (one 32-column panel, 32 X columns): k_gram32 gives
// each wave its own panel, so with one panel three of its four waves only stage X.  Here the
// four waves take consecutive 16-row slices of a 64-row chunk, load both operands straight
// from HBM (no LDS, no barrier in the loop; the next slice prefetched), and sum their tiles
// through LDS in wave order at the end (deterministic).  Same fp32 products; the per-split
// sum order differs from k_gram32 (rounding level).
template <int W>
__global__ __launch_bounds__(256) void k_gram32_one(int64_t nrows, const float* __restrict__ Wp,
                                                    const float* __restrict__ X,
                                                    double* __restrict__ slab, int64_t rows_per) {
  constexpr int T = W / 16;
  __shared__ f4v red[3][64][T * T];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int q = lane >> 4, c16 = lane & 15;
  const int64_t s = blockIdx.x;
  const int64_t r_begin = s * rows_per;
  const int64_t r_end = r_begin + rows_per < nrows ? r_begin + rows_per : nrows;
  f4v acc[T][T];
#pragma unroll
  for (int a = 0; a < T; ++a)
#pragma unroll
    for (int c = 0; c < T; ++c) acc[a][c] = f4v{0.f, 0.f, 0.f, 0.f};
  auto load = [&](int64_t rb, float (&ar)[4][T], float (&br)[4][T]) {
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      const int64_t row = rb + 4 * ks + q;
      const bool ok = row < r_end;
      const int64_t rr = ok ? row : (r_end > 0 ? r_end - 1 : 0);
#pragma unroll
      for (int a = 0; a < T; ++a) {
        const float av = Wp[rr * W + c16 + 16 * a];
        ar[ks][a] = ok ? av : 0.f;
        br[ks][a] = X[rr * W + c16 + 16 * a];
      }
    }
  };
  float ac[4][T], bc[4][T], an[4][T], bn[4][T];
  int64_t rb = r_begin + 16 * wave;
  if (r_begin < r_end) load(rb, ac, bc);
  for (; rb < r_end; rb += 64) {
    load(rb + 64, an, bn);  // clamped past the split: finite values met by zero A
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int a = 0; a < T; ++a)
#pragma unroll
        for (int c = 0; c < T; ++c) acc[a][c] = mfma16(ac[ks][a], bc[ks][c], acc[a][c]);
#pragma unroll
    for (int ks = 0; ks < 4; ++ks)
#pragma unroll
      for (int a = 0; a < T; ++a) {
        ac[ks][a] = an[ks][a];
        bc[ks][a] = bn[ks][a];
      }
  }
  if (wave > 0) {
#pragma unroll
    for (int a = 0; a < T; ++a)
#pragma unroll
      for (int c = 0; c < T; ++c) red[wave - 1][lane][a * T + c] = acc[a][c];
  }
  __syncthreads();
  if (wave != 0) return;
  double* out = slab + s * (int64_t)W * W;
#pragma unroll
  for (int a = 0; a < T; ++a)
#pragma unroll
    for (int c = 0; c < T; ++c) {
      f4v v = acc[a][c];
#pragma unroll
      for (int w = 0; w < 3; ++w) v += red[w][lane][a * T + c];
#pragma unroll
      for (int e = 0; e < 4; ++e) out[(int64_t)(16 * a + 4 * q + e) * W + 16 * c + c16] = (double)v[e];
    }
}

int gram32_splits(int64_t nrows) {
  int64_t s8 = 3 * window_grid() / 8;
  const int64_t max_s8 = (nrows + 8 * 128 - 1) / (8 * 128);
  if (s8 > max_s8) s8 = max_s8;
  if (s8 < 1) s8 = 1;
  return (int)(s8 * 8);
}

template <int W, int NX>
static void launch_gram32(int64_t nrows, const float* Wb, int64_t wstride, int nW, const float* X0,
                          const float* X1, double* slab, int splits, hipStream_t st) {
  const int npg = (nW + kG32Waves - 1) / kG32Waves;
  int64_t rows_per = (nrows + splits - 1) / splits;
  rows_per = (rows_per + kG32Rows - 1) / kG32Rows * kG32Rows;
  hipLaunchKernelGGL((k_gram32<W, NX>), dim3(npg * splits), dim3(256), 0, st, nrows, Wb, wstride,
                     nW, X0, X1, slab, npg, rows_per);
}

// ----------------------------------------------------------------------------------------
// Any panel width (mixed precision at b not in {16, 32}: C1's b = 8, the reference tests'
// b = 5): one thread per Gram entry and split, fp32 products accumulated in fp32 over the
// split's rows (sgemm's arithmetic), splits summed in fp64 by reduce_slab.
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_gram32_any(int64_t nrows, const float* __restrict__ Wb,
                                                    int64_t wstride, int nW, int w,
                                                    const float* __restrict__ X0,
                                                    const float* __restrict__ X1, int xcount,
                                                    double* __restrict__ slab, int64_t rows_per) {
  const int KW = nW * w, KC = xcount * w;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const int64_t s = blockIdx.y;
  if (e >= (int64_t)KW * KC) return;
  const int a = (int)(e / KC), c = (int)(e % KC);
  const float* wp = Wb + (int64_t)(a / w) * wstride + (a % w);
  const float* xp = (c < w ? X0 : X1) + (c % w);
  const int64_t r0 = s * rows_per, r1 = r0 + rows_per < nrows ? r0 + rows_per : nrows;
  float acc = 0.f;
  for (int64_t r = r0; r < r1; ++r) acc = fmaf(wp[r * w], xp[r * w], acc);
  slab[s * KW * KC + e] = (double)acc;
}

// Y = beta Y + alpha X C at any width: one thread per element of Y (Y must not alias X)
__global__ __launch_bounds__(256) void k_tsmm32_any(int64_t nrows, const float* __restrict__ Xb,
                                                    int64_t xstride, int nX, int w,
                                                    const double* __restrict__ C, int ldc,
                                                    float* Y0, float* Y1, int ycount, float alpha,
                                                    float beta) {
  const int KY = ycount * w, K = nX * w;
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= nrows * KY) return;
  const int64_t r = e / KY;
  const int c = (int)(e % KY);
  float acc = 0.f;
  for (int k = 0; k < K; ++k)
    acc = fmaf(Xb[(int64_t)(k / w) * xstride + r * w + (k % w)], (float)C[(int64_t)k * ldc + c], acc);
  float* y = (c < w ? Y0 : Y1) + r * w + (c % w);
  *y = beta != 0.f ? beta * *y + alpha * acc : alpha * acc;
}

// RBL_LOC32_MFMA=1 (variants build only): the fp32-basis local reorth on the MFMA tile
// kernels instead of the 4-wave Gram / row-streaming update (A/B)
#ifdef RBL_VARIANTS
static bool loc32_mfma() { return std::getenv("RBL_LOC32_MFMA") != nullptr; }
#else
static constexpr bool loc32_mfma() { return false; }
#endif

void gram32_partial(int64_t nrows, const float* Wb, int64_t wstride, int nW, int w, const float* X0,
                    const float* X1, int xcount, double* slab, int splits, hipStream_t st) {
  if (w != 16 && w != 32) {
    const int64_t len = (int64_t)nW * w * xcount * w;
    const int64_t rows_per = (nrows + splits - 1) / splits;
    hipLaunchKernelGGL(k_gram32_any, dim3((unsigned)((len + 255) / 256), (unsigned)splits), dim3(256), 0,
                       st, nrows, Wb, wstride, nW, w, X0, X1, xcount, slab, rows_per);
    return;
  }
  if (w == 32 && nW == 1 && xcount == 1 && !loc32_mfma()) {
    int64_t rows_per = (nrows + splits - 1) / splits;
    rows_per = (rows_per + 63) / 64 * 64;
    hipLaunchKernelGGL(k_gram32_one<32>, dim3((unsigned)splits), dim3(256), 0, st, nrows, Wb, X0, slab,
                       rows_per);
    return;
  }
  if (w == 32) {
    if (xcount == 2 && RBL_G32_MFMA32) {
      const int npg = (nW + kG32Waves - 1) / kG32Waves;
      int64_t rows_per = (nrows + splits - 1) / splits;
      rows_per = (rows_per + kG32Rows - 1) / kG32Rows * kG32Rows;
      hipLaunchKernelGGL(k_gram32x, dim3(npg * splits), dim3(256), 0, st, nrows, Wb, wstride, nW, X0, X1,
                         slab, npg, rows_per);
      return;
    }
    if (xcount == 2) return launch_gram32<32, 2>(nrows, Wb, wstride, nW, X0, X1, slab, splits, st);
    return launch_gram32<32, 1>(nrows, Wb, wstride, nW, X0, X1, slab, splits, st);
  }
  if (xcount == 2) return launch_gram32<16, 2>(nrows, Wb, wstride, nW, X0, X1, slab, splits, st);
  return launch_gram32<16, 1>(nrows, Wb, wstride, nW, X0, X1, slab, splits, st);
}

// ----------------------------------------------------------------------------------------
// Y = beta Y + alpha X C (fp32): 4 waves x 32 rows per workgroup; C (fp64 Gram, rounded to
// f32 as the reference's FLOAT temp) staged in LDS 16 k at a time as k * 64 + 4 (c & 15) +
// (c >> 4); A operands one float4 per lane per row tile covering 4 k-steps (k permuted:
// lane quarter q takes k = k0 + 4q + s in step s, matched on the C side).
// ----------------------------------------------------------------------------------------
constexpr int kT32Rows = 32;  // rows per wave
constexpr int kT32K = 16;     // k per chunk

template <int W, int KYP>
__global__ __launch_bounds__(256) void k_tsmm32(int64_t nrows, const float* __restrict__ Xb,
                                                int64_t xstride, int nX, const double* __restrict__ C,
                                                int ldc, int KY, float* Y0, float* Y1, float alpha,
                                                float beta) {
  constexpr int CT = KYP / 16;
  __shared__ __attribute__((aligned(16))) float cs[2][kT32K * 64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, c16 = lane & 15;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * kT32Rows;
  const int K = nX * W;
  const int nch = (K + kT32K - 1) / kT32K;

  f4v acc[2][CT];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[rt][c] = f4v{0.f, 0.f, 0.f, 0.f};

  int64_t arow[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int64_t r = r0 + 16 * rt + c16;
    arow[rt] = r < nrows ? r : nrows - 1;
  }
  auto load_a = [&](int ch, f4v (&ar)[2]) {
    const int k0 = ch * kT32K + 4 * q;
    const int k = k0 < K ? k0 : K - 4;  // clamped: k past K meets zero C rows
    const int pan = k / W, col = k - pan * W;
    const float* xp = Xb + (int64_t)pan * xstride + col;
#pragma unroll
    for (int rt = 0; rt < 2; ++rt) ar[rt] = *reinterpret_cast<const f4v*>(xp + arow[rt] * W);
  };
  // C chunk: 16 x KYP; thread (k = tid / 16, cc = tid % 16) moves C[k][cc + 16 ct]
  const int ck = tid >> 4, ccc = tid & 15;
  auto load_c = [&](int ch, float (&cr)[CT]) {
    const int k = ch * kT32K + ck;
    const int kc = k < K ? k : K - 1;
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) {
      const int c = ccc + 16 * ct;
      const int cc = c < KY ? c : KY - 1;
      const float v = (float)C[(int64_t)kc * ldc + cc];
      cr[ct] = (k < K && c < KY) ? alpha * v : 0.f;
    }
  };
  auto store_c = [&](int buf, const float (&cr)[CT]) {
    float* d = &cs[buf][ck * 64 + 4 * ccc];
#pragma unroll
    for (int ct = 0; ct < CT; ++ct) d[ct] = cr[ct];
  };

  f4v acur[2], anext[2];
  float cr[CT];
  load_c(0, cr);
  store_c(0, cr);
  load_a(0, acur);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    load_c(ch + 1, cr);
    load_a(ch + 1, anext);
    const float* cb = cs[ch & 1] + 4 * c16;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const f4v bv = *reinterpret_cast<const f4v*>(cb + (4 * q + s) * 64);
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
#pragma unroll
        for (int c = 0; c < CT; ++c) acc[rt][c] = mfma16(acur[rt][s], bv[c], acc[rt][c]);
    }
    store_c((ch + 1) & 1, cr);
    acur[0] = anext[0];
    acur[1] = anext[1];
    __syncthreads();
  }
  // D: lane holds rows 4q + v, column c16 of tile (rt, c): 64-B row segments
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int c = 0; c < CT; ++c) {
      const int col = 16 * c + c16;
      if (col >= KY) continue;
      float* yp = col < W ? Y0 + col : Y1 + (col - W);
#pragma unroll
      for (int v = 0; v < 4; ++v) {
        const int64_t r = r0 + 16 * rt + 4 * q + v;
        if (r < nrows) {
          float y = acc[rt][c][v];
          if (beta != 0.f) y += beta * yp[r * W];
          yp[r * W] = y;
        }
      }
    }
}

// Fast path of k_tsmm32 for the partial-reorth update (W = 32, 64 output columns, K a
// multiple of 32, nrows >= 32): 32 k per chunk (half the barriers), wave-uniform bases plus
// lane constants (no per-load clamps), a wave past nrows computes the last 32 rows and stores
// only its own, 16-B Y stores through the wave's LDS tile.
// KF: k per chunk (one barrier per 2 KF MFMAs per wave), 32 or 64 (two basis panels; even nX).
// 64 measured 1.5 % slower (occupancy 5 -> 4; profiles/r03_tsmm32_kf_ab.log), so 32
#ifndef RBL_T32_KF
#define RBL_T32_KF 32
#endif
template <int KF>
__global__ __launch_bounds__(256) void k_tsmm32f(int64_t nrows, const float* __restrict__ Xb,
                                                 int64_t xstride, int nX, const double* __restrict__ C,
                                                 int ldc, float* Y0, float* Y1, float alpha,
                                                 float beta) {
  constexpr int W = 32, KYP = 64, CT = 4, CLD = 64;
  constexpr int kT32KF = KF, HH = KF / 16;
  // two C buffers; after the k-loop the same LDS holds the 4 waves' 16 x (64 + 4) Y tiles
  __shared__ __attribute__((aligned(16))) float cs[2][kT32KF * CLD + 128];
  static_assert(2 * (kT32KF * CLD + 128) >= 4 * 16 * (KYP + 4), "epilogue tiles fit");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4, c16 = lane & 15;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * kT32Rows;
  const int64_t rw = r0 + kT32Rows <= nrows ? r0 : nrows - kT32Rows;  // wave-uniform
  const int nch = nX * W / kT32KF;

  f4v acc[2][CT];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int c = 0; c < CT; ++c) acc[rt][c] = f4v{0.f, 0.f, 0.f, 0.f};

  // A: rows rw + 16 rt + c16; k = KF ch + 16 hh + 4 q + s (one float4 per (rt, hh)); the
  // chunk spans KF / 32 basis panels (hh / 2 selects the panel at KF = 64)
  const int aoff = c16 * W + 4 * q;
  auto load_a = [&](int ch, f4v (&ar)[2][HH]) {
    const int chc = ch < nch ? ch : nch - 1;
#pragma unroll
    for (int hh = 0; hh < HH; ++hh) {
      const float* xb = Xb + (int64_t)(KF / W * chc + hh / 2) * xstride + rw * W;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt)
        ar[rt][hh] = *reinterpret_cast<const f4v*>(xb + aoff + 16 * rt * W + 16 * (hh & 1));
    }
  };
  // C chunk: KF x 64; thread (k = tid / 16 + 16 hh, cc = tid % 16) moves C[k][cc + 16 ct]
  const int ck = tid >> 4, ccc = tid & 15;
  auto load_c = [&](int ch, float (&cr)[HH][CT]) {
    const int chc = ch < nch ? ch : nch - 1;
    const double* cb = C + (int64_t)(kT32KF * chc + ck) * ldc + ccc;
#pragma unroll
    for (int hh = 0; hh < HH; ++hh)
#pragma unroll
      for (int ct = 0; ct < CT; ++ct) cr[hh][ct] = alpha * (float)cb[(int64_t)(16 * hh) * ldc + 16 * ct];
  };
  auto store_c = [&](int buf, const float (&cr)[HH][CT]) {
#pragma unroll
    for (int hh = 0; hh < HH; ++hh)
      *reinterpret_cast<f4v*>(&cs[buf][(ck + 16 * hh) * CLD + 4 * ccc]) =
          f4v{cr[hh][0], cr[hh][1], cr[hh][2], cr[hh][3]};
  };

  f4v acur[2][HH], anext[2][HH];
  float cr[HH][CT];
  load_c(0, cr);
  store_c(0, cr);
  load_a(0, acur);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    load_c(ch + 1, cr);
    load_a(ch + 1, anext);
    const float* cb = cs[ch & 1] + 4 * c16;
#pragma unroll
    for (int hh = 0; hh < HH; ++hh)
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const f4v bv = *reinterpret_cast<const f4v*>(cb + (16 * hh + 4 * q + s) * CLD);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
          for (int c = 0; c < CT; ++c) acc[rt][c] = mfma16(acur[rt][hh][s], bv[c], acc[rt][c]);
      }
    store_c((ch + 1) & 1, cr);
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int hh = 0; hh < HH; ++hh) acur[rt][hh] = anext[rt][hh];
    __syncthreads();
  }
  // epilogue: D tile (lane: rows 4q + v, column c16 of tile c) -> LDS (free after the last
  // barrier) -> row-major float4 stores of Y0 | Y1 (rows below r0: the previous wave's)
  float* ot = &cs[0][0] + wave * 16 * (KYP + 4);
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
#pragma unroll
    for (int c = 0; c < CT; ++c)
#pragma unroll
      for (int v = 0; v < 4; ++v) ot[(4 * q + v) * (KYP + 4) + 16 * c + c16] = acc[rt][c][v];
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int e = 4 * lane + 256 * m, row = e / KYP, col = e % KYP;
      const int64_t r = rw + 16 * rt + row;
      f4v y = *reinterpret_cast<const f4v*>(ot + row * (KYP + 4) + col);
      if (r >= r0 && r < nrows) {
        float* yp = (col < W ? Y0 + col : Y1 + (col - W)) + r * W;
        if (beta != 0.f) y += beta * *reinterpret_cast<const f4v*>(yp);
        *reinterpret_cast<f4v*>(yp) = y;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

// The partial-reorth update on v_mfma_f32_32x32x2f32 (W = 32, 64 output columns): a wave owns
// 32 rows (one 32 x 32 tile per output panel).  Step s of a 32-k chunk (one basis panel) takes
// k = s for lanes 0-31 and k = 16 + s for lanes 32-63, so lane l loads its row's 16
// consecutive k once per chunk (four float4: row rw + l % 32, k 16 (l / 32) ..) and B[k][j] =
// alpha C[k][j] (+32 for the second panel) sits pairwise in LDS (row k, column c at
// k * 64 + 2 (c % 32) + c / 32): one ds_read_b64 per step feeds both tiles.  Epilogue as
// k_tsmm32f, by 16-row halves (registers v < 8 hold rows 0-15 of the tile).
#ifndef RBL_T32_MFMA32
#define RBL_T32_MFMA32 1
#endif
#ifndef RBL_T32X_PINGPONG
#define RBL_T32X_PINGPONG 0
#endif
__global__ __launch_bounds__(256) void k_tsmm32x(int64_t nrows, const float* __restrict__ Xb,
                                                 int64_t xstride, int nX, const double* __restrict__ C,
                                                 int ldc, float* Y0, float* Y1, float alpha,
                                                 float beta) {
  constexpr int W = 32, KYP = 64, KF = 32, NS = 16, CLD = 64;
  __shared__ __attribute__((aligned(16))) float cs[2][KF * CLD + 128];
  static_assert(2 * (KF * CLD + 128) >= 4 * 16 * (KYP + 4), "epilogue tiles fit");
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * kT32Rows;
  const int64_t rw = r0 + kT32Rows <= nrows ? r0 : nrows - kT32Rows;  // wave-uniform
  const int nch = nX;  // one 32-column basis panel per chunk

  f16v acc[2];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt)
#pragma unroll
    for (int v = 0; v < 16; ++v) acc[tt][v] = 0.f;

  const unsigned aoff = (unsigned)((lane % 32) * W + 16 * (lane / 32));
  auto load_a = [&](int ch, f4v (&ar)[4]) {
    const int chc = ch < nch ? ch : nch - 1;
    const float* xb = Xb + (int64_t)chc * xstride + rw * W;  // uniform
#pragma unroll
    for (int u = 0; u < 4; ++u) ar[u] = *reinterpret_cast<const f4v*>(xb + (aoff + 4u * u));
  };
  // C chunk 32 x 64: thread (k = tid / 8, c0 = 4 (tid % 8)) moves C[k][c0 .. c0 + 3] and
  // C[k][32 + c0 .. 32 + c0 + 3] into 8 consecutive floats (pairwise interleaved)
  const int ck = tid >> 3, cc0 = 4 * (tid & 7);
  auto load_c = [&](int ch, float (&cr)[8]) {
    const int chc = ch < nch ? ch : nch - 1;
    const double* cb = C + (int64_t)(KF * chc + ck) * ldc + cc0;
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      cr[2 * u] = alpha * (float)cb[u];
      cr[2 * u + 1] = alpha * (float)cb[W + u];
    }
  };
  auto store_c = [&](int buf, const float (&cr)[8]) {
    float* d = &cs[buf][ck * CLD + 2 * cc0];
    *reinterpret_cast<f4v*>(d) = f4v{cr[0], cr[1], cr[2], cr[3]};
    *reinterpret_cast<f4v*>(d + 4) = f4v{cr[4], cr[5], cr[6], cr[7]};
  };

  f4v acur[4], anext[4];
  float cr[8];
  load_c(0, cr);
  store_c(0, cr);
  load_a(0, acur);
  __syncthreads();
  // one chunk: MFMAs on `use` while chunk ch + 1's operands land in `pf`
  auto chunk = [&](int ch, const f4v (&use)[4], f4v (&pf)[4]) {
    load_c(ch + 1, cr);
    load_a(ch + 1, pf);
    const float* cb = cs[ch & 1] + 16 * (lane / 32) * CLD + 2 * (lane % 32);
#pragma unroll
    for (int st = 0; st < NS; ++st) {
      const float2 bv = *reinterpret_cast<const float2*>(cb + st * CLD);
      const float a = use[st / 4][st % 4];
      acc[0] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv.x, acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv.y, acc[1], 0, 0, 0);
    }
    store_c((ch + 1) & 1, cr);
    __syncthreads();
  };
#if RBL_T32X_PINGPONG
  // chunks in pairs with the two operand sets swapping roles: no register rotation per chunk
  // (16 v_mov per 32 MFMAs in the rotating form; VALU per MFMA 1.2 -> 0.67 in the loop), but
  // measured 5 % slower (partial reorth 288 vs 274 ms per fp32 C4a run, 3 alternating
  // reps, profiles/r04_t32pp_ab.log: the 64-MFMA loop body), so off
  for (int ch = 0; ch < nch; ch += 2) {
    chunk(ch, acur, anext);
    if (ch + 1 < nch) chunk(ch + 1, anext, acur);  // (wave-uniform)
  }
#else
  for (int ch = 0; ch < nch; ++ch) {
    chunk(ch, acur, anext);
#pragma unroll
    for (int u = 0; u < 4; ++u) acur[u] = anext[u];
  }
#endif
  // epilogue: D (lane l, register v: row 4 (l / 32) + v % 4 + 8 (v / 4), column l % 32 of tile
  // tt) -> LDS by 16-row halves -> row-major float4 stores of Y0 | Y1 (rows below r0: the
  // previous wave's)
  float* ot = &cs[0][0] + wave * 16 * (KYP + 4);
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
#pragma unroll
    for (int tt = 0; tt < 2; ++tt)
#pragma unroll
      for (int v = 8 * rt; v < 8 * rt + 8; ++v) {
        const int i = 4 * (lane / 32) + (v % 4) + 8 * (v / 4) - 16 * rt;
        ot[i * (KYP + 4) + W * tt + (lane % 32)] = acc[tt][v];
      }
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
    for (int m = 0; m < 4; ++m) {
      const int e = 4 * lane + 256 * m, row = e / KYP, col = e % KYP;
      const int64_t r = rw + 16 * rt + row;
      f4v y = *reinterpret_cast<const f4v*>(ot + row * (KYP + 4) + col);
      if (r >= r0 && r < nrows) {
        float* yp = (col < W ? Y0 + col : Y1 + (col - W)) + r * W;
        if (beta != 0.f) y += beta * *reinterpret_cast<const f4v*>(yp);
        *reinterpret_cast<f4v*>(yp) = y;
      }
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
}

template <int W, int KYP>
static void launch_tsmm32(int64_t nrows, const float* Xb, int64_t xstride, int nX, const double* C,
                          int ldc, int KY, float* Y0, float* Y1, float alpha, float beta,
                          hipStream_t st) {
  const int64_t wgs = (nrows + 4 * kT32Rows - 1) / (4 * kT32Rows);
  hipLaunchKernelGGL((k_tsmm32<W, KYP>), dim3((unsigned)wgs), dim3(256), 0, st, nrows, Xb, xstride,
                     nX, C, ldc, KY, Y0, Y1, alpha, beta);
}

// Y += alpha X C for ONE 32-column panel X and 32 output columns (the fp32 local reorth,
// Q_i -= Q_{i-1} (Q_{i-1}^T Q_i), RBL_gpu.jl:83-93 in FLOAT): a streaming pass, so lanes move
// whole rows instead of MFMA tiles.  Per 32-row group the workgroup reads X and Y as one
// contiguous 4 KiB float4 each (thread t: quad t % 8 of row t / 8); X goes through LDS so each
// lane sees its row, Y stays in the lane's register.  The grid is persistent (C staged once per
// workgroup as alpha * fp32(C), as k_tsmm32).  The sum runs in k_tsmm32's MFMA order (chunk of
// 16 k, step s, lane quarter q: k = 16 ch + 4 q + s) as an fmaf chain, then adds Y: the same
// bits as that kernel (tested).
__global__ __launch_bounds__(256) void k_upd32_rows(int64_t nrows, const float* __restrict__ X,
                                                    const double* __restrict__ C, int ldc,
                                                    float* __restrict__ Y, float alpha) {
  __shared__ __attribute__((aligned(16))) float cs[32 * 32];
  __shared__ f4v xs[2][256];
  for (int i = threadIdx.x; i < 32 * 32; i += 256)
    cs[i] = alpha * (float)C[(int64_t)(i >> 5) * ldc + (i & 31)];
  const int t = threadIdx.x, j = t & 7, row = t >> 3;
  const int64_t ngroups = (nrows + 31) / 32;
  const f4v* X4 = reinterpret_cast<const f4v*>(X);
  f4v* Y4 = reinterpret_cast<f4v*>(Y);
  int buf = 0;
  for (int64_t g = blockIdx.x; g < ngroups; g += gridDim.x, buf ^= 1) {
    const int64_t e = g * 256 + t;             // float4 index: row g * 32 + row, quad j
    const bool ok = g * 32 + row < nrows;
    xs[buf][t] = ok ? X4[e] : f4v{0.f, 0.f, 0.f, 0.f};
    f4v y = ok ? Y4[e] : f4v{0.f, 0.f, 0.f, 0.f};
    __syncthreads();                           // (two buffers: one barrier per group)
    const f4v* xr = &xs[buf][row * 8];
    float x[32];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const f4v v = xr[i];
      x[4 * i] = v[0];
      x[4 * i + 1] = v[1];
      x[4 * i + 2] = v[2];
      x[4 * i + 3] = v[3];
    }
    f4v acc = f4v{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int s = 0; s < 4; ++s)
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int k = 16 * ch + 4 * q + s;
          const f4v c = *reinterpret_cast<const f4v*>(cs + 32 * k + 4 * j);
#pragma unroll
          for (int m = 0; m < 4; ++m) acc[m] = fmaf(x[k], c[m], acc[m]);
        }
#pragma unroll
    for (int m = 0; m < 4; ++m) y[m] = acc[m] + y[m];
    if (ok) Y4[e] = y;
  }
}

void tsmm32(int64_t nrows, const float* Xb, int64_t xstride, int nX, int w, const double* C, int ldc,
            float* Y0, float* Y1, int ycount, float alpha, float beta, hipStream_t st) {
  if (nrows <= 0) return;
  const int KY = ycount * w;
  // the local reorth's shape (one panel, 32 columns, Y += X C); RBL_LOC32_MFMA=1: the tile kernel
  if (w == 32 && nX == 1 && KY == 32 && beta == 1.f && !loc32_mfma()) {
    const int64_t groups = (nrows + 31) / 32;
    const int64_t grid = groups < 8 * (int64_t)window_grid() ? groups : 8 * (int64_t)window_grid();
    hipLaunchKernelGGL(k_upd32_rows, dim3((unsigned)grid), dim3(256), 0, st, nrows, Xb, C, ldc, Y0, alpha);
    return;
  }
  if (w != 16 && w != 32) {
    const int64_t thr = nrows * KY;
    hipLaunchKernelGGL(k_tsmm32_any, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, st, nrows, Xb,
                       xstride, nX, w, C, ldc, Y0, Y1, ycount, alpha, beta);
    return;
  }
  if (w == 32 && KY == 64 && nrows >= kT32Rows) {
    const int64_t wgs = (nrows + 4 * kT32Rows - 1) / (4 * kT32Rows);
    if (RBL_T32_MFMA32) {
      hipLaunchKernelGGL(k_tsmm32x, dim3((unsigned)wgs), dim3(256), 0, st, nrows, Xb, xstride, nX, C,
                         ldc, Y0, Y1, alpha, beta);
      return;
    }
    if (RBL_T32_KF == 64 && nX % 2 == 0)
      hipLaunchKernelGGL(k_tsmm32f<64>, dim3((unsigned)wgs), dim3(256), 0, st, nrows, Xb, xstride, nX, C,
                         ldc, Y0, Y1, alpha, beta);
    else
      hipLaunchKernelGGL(k_tsmm32f<32>, dim3((unsigned)wgs), dim3(256), 0, st, nrows, Xb, xstride, nX, C,
                         ldc, Y0, Y1, alpha, beta);
    return;
  }
  if (w == 32) {
    if (KY <= 32) return launch_tsmm32<32, 32>(nrows, Xb, xstride, nX, C, ldc, KY, Y0, Y1, alpha, beta, st);
    return launch_tsmm32<32, 64>(nrows, Xb, xstride, nX, C, ldc, KY, Y0, Y1, alpha, beta, st);
  }
  if (KY <= 16) return launch_tsmm32<16, 16>(nrows, Xb, xstride, nX, C, ldc, KY, Y0, Y1, alpha, beta, st);
  return launch_tsmm32<16, 32>(nrows, Xb, xstride, nX, C, ldc, KY, Y0, Y1, alpha, beta, st);
}

// ---- conversions -------------------------------------------------------------------------
// element-wise conversions for blocks whose slot offset is not 16-B aligned (b odd)
__global__ void k_f32_to_f64_s(const float* __restrict__ src, double* __restrict__ dst, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = src[i];
}
__global__ void k_f64_to_f32_s(const double* __restrict__ src, float* __restrict__ dst, int64_t n) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) dst[i] = (float)src[i];
}
static bool aligned16(const void* a, const void* b) {
  return (((uintptr_t)a | (uintptr_t)b) & 15) == 0;
}
__global__ void k_f32_to_f64(const float* __restrict__ src, double* __restrict__ dst, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n) {
    const f4v v = *reinterpret_cast<const f4v*>(src + i);
    *reinterpret_cast<d2v*>(dst + i) = d2v{v.x, v.y};
    *reinterpret_cast<d2v*>(dst + i + 2) = d2v{v.z, v.w};
  } else {
    for (int64_t e = i; e < n; ++e) dst[e] = src[e];
  }
}
__global__ void k_f64_to_f32(const double* __restrict__ src, float* __restrict__ dst, int64_t n) {
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) * 4;
  if (i + 3 < n) {
    const d2v a = *reinterpret_cast<const d2v*>(src + i), b = *reinterpret_cast<const d2v*>(src + i + 2);
    *reinterpret_cast<f4v*>(dst + i) = f4v{(float)a.x, (float)a.y, (float)b.x, (float)b.y};
  } else {
    for (int64_t e = i; e < n; ++e) dst[e] = (float)src[e];
  }
}
void cvt_f32_to_f64(const float* src, double* dst, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  if (!aligned16(src, dst)) {
    hipLaunchKernelGGL(k_f32_to_f64_s, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, dst, n);
    return;
  }
  const int64_t thr = (n + 3) / 4;
  hipLaunchKernelGGL(k_f32_to_f64, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, s, src, dst, n);
}
void cvt_f64_to_f32(const double* src, float* dst, int64_t n, hipStream_t s) {
  if (n <= 0) return;
  if (!aligned16(src, dst)) {
    hipLaunchKernelGGL(k_f64_to_f32_s, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, src, dst, n);
    return;
  }
  const int64_t thr = (n + 3) / 4;
  hipLaunchKernelGGL(k_f64_to_f32, dim3((unsigned)((thr + 255) / 256)), dim3(256), 0, s, src, dst, n);
}

}  // namespace rbl
