// rowop.hip — fused b x b row operations of the block step on v_mfma_f64_4x4x4f64 (gfx950):
//
//   Y' = beta Y + alpha X C          (X, Y: n x B panels, C: B x B)
//   G  = Y'^T Y'   (optional)        (per-workgroup partials, reduced by reduce_slab)
//
// One pass over X and Y instead of two: the 3-term update U -= Q_i A_i (RBL_gpu.jl:179)
// hands CholQR its first Gram U^T U, and each CholQR apply Q = U R^-1 (RBL_gpu.jl:180) the
// Gram of the next pass (tsqr in rbl_api.cpp).
//
// The Gram needs no data movement: in the MFMA D layout a lane holds
// Y'[4g + (lane>>4)][4cg + (lane&3)] for row quad g = (lane>>2)&3 and column group cg, which
// is exactly the A operand (A[i = lane&3][k = lane>>4] = Y'[k][4icg + i]) and the B operand
// (B[k = lane>>4][j = lane&3] = Y'[k][4jcg + j]) of the 4x4x4 MFMA whose block g yields
// sum_{k in quad g} Y'[k][4icg + i] Y'[k][4jcg + j]; the four blocks are summed once at the end.
//
// Two more forms serve CholQR2 with one pass fewer (tsqr in rbl_api.cpp):
//   MODE 1: G = (X C)^T (X C) only (no store): pass 1 of CholQR2 forms the Gram of Q1 = U R1^-1
//           without writing Q1;
//   MODE 2: Y' = (X C) C2: pass 2 recomputes Q1 = U R1^-1 bit for bit (same operands, same
//           MFMA order) and applies R2^-1 in the same pass, so Q1 never goes to HBM (3 passes
//           over n x b per QR instead of 4; the same bits as the 4-pass form).
// TRI: C (and C2) upper triangular (CholQR's R^-1): an MFMA whose four k rows of C are all
// zero in its four columns (k > c throughout) adds exact zeros and is skipped — 24 of the 64
// per 16-row tile at b = 32 (the k-interleave 8h + 2q + v keeps the order of every other MFMA).
// XG: the cross Gram Z^T Y' of another block Z (v_mfma_f64_16x16x4f64, Z read in its A layout,
// Y' from the output stage): the next step's local-reorth coefficient Q_{i}^T Q_{i+1}
// (RBL_gpu.jl:87) formed while Q_{i+1} is written.
//
// Persistent grid: each wave walks 16-row tiles grid-stride (register budget), with the next
// block's X (A layout, 16 B per lane) and Y (row-major, 16 B per lane) prefetched.  Y enters
// and leaves the D layout through a per-wave LDS tile (column c of row r stored at
// c ^ 4((r >> 2) & 3): the four row quads of a ds_write_b64 lane group land 8 banks apart).
#include <atomic>

#include "kernels.hpp"

namespace rbl {

namespace {

constexpr int kRowThreads = 256;  // 4 waves
// minimum waves per SIMD asked of the compiler: the Gram / cross-Gram forms, the others.
// Four waves for CholQR2's Gram-only pass (132 -> 126 VGPRs) and the plain row update (130 ->
// 126) measured ~2 % slower on both (qr 71.5 -> 73.0 ms per C4a run, R-MAT loc reorth 51.5 ->
// 52.5 ms; profiles/r03_rowop_wpe4_ab.log): these MFMA-heavy streams prefer fewer waves
#ifndef RBL_RG_WPE_G
#define RBL_RG_WPE_G 2
#endif
#ifndef RBL_RG_WPE
#define RBL_RG_WPE 3
#endif
#ifndef RBL_RG_WPE_M1  // MODE 1 (CholQR2's Gram-only pass)
#define RBL_RG_WPE_M1 RBL_RG_WPE_G
#endif
constexpr int kBlockRows = 16;    // rows per wave per iteration (one MFMA row tile)

typedef double d4v __attribute__((ext_vector_type(4)));
__device__ __forceinline__ double mfma4r(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
// n x b blocks are streamed once per pass (2.56 GB at C4a, far beyond L2 + Infinity Cache):
// non-temporal loads and stores (RBL_ROWOP_NT=0 restores the default policy for A/B runs)
#ifndef RBL_ROWOP_NT
#define RBL_ROWOP_NT 1
#endif
__device__ __forceinline__ d2v ldnt(const d2v* p) {
  if constexpr (RBL_ROWOP_NT) return __builtin_nontemporal_load(p);
  return *p;
}
__device__ __forceinline__ void stnt(d2v v, d2v* p) {
  if constexpr (RBL_ROWOP_NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// acc[cg] += a * C[k][4cg + j] for the k rows k0 + 2q (q = 0..3) of one MFMA, columns in perm8
// order (column groups 2cp, 2cp+1 in one 16-B read); TRI: column groups with 4cg + 3 < k0 are
// all zero in C and skipped (compile-time: k0 and cg are unrolled constants)
template <bool TRI, int CG>
__device__ __forceinline__ void mfma_row(const int k0, double a, const double* cb, double (&acc)[CG]) {
#pragma unroll
  for (int cp = 0; cp < CG / 2; ++cp) {
    const bool z0 = TRI && k0 > 8 * cp + 3, z1 = TRI && k0 > 8 * cp + 7;
    if (z0 && z1) continue;
    const d2v bf = *reinterpret_cast<const d2v*>(cb + 8 * cp);
    if (!z0) acc[2 * cp] = mfma4r(a, bf.x, acc[2 * cp]);
    if (!z1) acc[2 * cp + 1] = mfma4r(a, bf.y, acc[2 * cp + 1]);
  }
  if constexpr (CG % 2) {
    if (!(TRI && k0 > 4 * (CG - 1) + 3)) acc[CG - 1] = mfma4r(a, cb[8 * (CG / 2)], acc[CG - 1]);
  }
}

// XF: X is read from X32 (fp32, widened exactly); YF: Y' goes to Y32 rounded to fp32 (as
// cvt_f64_to_f32) unless *f64flag is set, then to Y in fp64 — the fp32-basis step's QR
// (RBL_gpu.jl:182 `Qg = FLOAT(Qg_d)`) without a separate narrowing pass.
template <int B, bool GRAM, bool XF = false, bool YF = false, int MODE = 0, bool XG = false,
          bool TRI = false>
__global__ __launch_bounds__(kRowThreads) __attribute__((amdgpu_waves_per_eu(MODE == 1 ? RBL_RG_WPE_M1 : GRAM || XG ? RBL_RG_WPE_G : RBL_RG_WPE))) void k_rowgram(int64_t nrows, const double* X,  // X may alias Y (in-place apply)
                                                         const double* __restrict__ C, int ldc,
                                                         double* Y, double alpha, double beta,
                                                         double* __restrict__ slab, const int* skip,
                                                         const float* X32, float* Y32,
                                                         const int* f64flag, const double* __restrict__ C2,
                                                         const double* __restrict__ Z,
                                                         double* __restrict__ slab2) {
  if (skip && *skip) return;
  constexpr bool TWO = MODE == 2, STORE = MODE != 1;
  const bool w64 = !YF || (f64flag && *f64flag);
  constexpr int CG = B / 4;
  constexpr int NH = B / 8;                 // A-operand loads per row tile (2 k each)
  constexpr int LDC = B + 8;                // C rows: lane-group rows differ by 2 (see reorth.hip)
  constexpr int kYPer = 16 * B / 128;       // row-major d2v per lane per 16-row tile
  constexpr int NG = CG * (CG + 1) / 2;     // Gram accumulators (upper triangle of quads)
  constexpr int NT = B / 16;                // 16-column tiles of the cross Gram
  // LDS: alpha C | C2 (MODE 2) | the waves' output stages; the end-of-kernel Gram reductions
  // reuse all of it
  constexpr int kMain = B * LDC + (TWO ? B * LDC : 0) + 4 * 16 * B;
  constexpr int kRed = GRAM || XG ? 4 * B * B : 0;
  __shared__ __attribute__((aligned(16))) double lds[kMain > kRed ? kMain : kRed];
  double* cs = lds;
  double* cs2 = lds + B * LDC;
  double* gs = lds;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4, g = (lane >> 2) & 3, j = lane & 3;

  // alpha C into LDS, columns in perm8 order (column groups 2cp, 2cp+1 in one 16-B read)
  for (int e = tid; e < B * B; e += kRowThreads) {
    const int k = e / B, c = e % B;
    cs[k * LDC + perm8(c)] = alpha * C[(int64_t)k * ldc + c];
    if constexpr (TWO) cs2[k * LDC + perm8(c)] = C2[(int64_t)k * ldc + c];
  }
  __syncthreads();

  double* ot = lds + B * LDC + (TWO ? B * LDC : 0) + wave * 16 * B;
  auto swz = [](int row, int c) { return row * B + (c ^ (4 * ((row >> 2) & 3))); };

  const int64_t nblk = (nrows + kBlockRows - 1) / kBlockRows;
  const int64_t stride = (int64_t)gridDim.x * 4;
  int64_t blk = (int64_t)blockIdx.x * 4 + wave;

  // loads (clamped rows: always issued)
  auto load_x = [&](int64_t b0, d2v (&xa)[1][NH]) {
#pragma unroll
    for (int rt = 0; rt < 1; ++rt) {
      int64_t r = b0 * kBlockRows + 16 * rt + (lane & 15);
      r = r < nrows ? r : nrows - 1;
#pragma unroll
      for (int h = 0; h < NH; ++h)
        if constexpr (XF) {
          const float2 f = *reinterpret_cast<const float2*>(X32 + r * B + 8 * h + 2 * q);
          xa[rt][h] = d2v{(double)f.x, (double)f.y};
        } else {
          xa[rt][h] = ldnt(reinterpret_cast<const d2v*>(X + r * B + 8 * h + 2 * q));
        }
    }
  };
  auto load_y = [&](int64_t b0, d2v (&yr)[1][kYPer]) {
#pragma unroll
    for (int rt = 0; rt < 1; ++rt)
#pragma unroll
      for (int m = 0; m < kYPer; ++m) {
        const int e = 2 * lane + 128 * m;
        int64_t r = b0 * kBlockRows + 16 * rt + e / B;
        r = r < nrows ? r : nrows - 1;
        yr[rt][m] = ldnt(reinterpret_cast<const d2v*>(Y + r * B + (e % B)));
      }
  };

  // Z in the 16x16x4 A layout: za[s][it] = Z[16 blk + 4 s + q][16 it + (lane & 15)]
  auto load_z = [&](int64_t b0, double (&za)[4][NT]) {
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      int64_t r = b0 * kBlockRows + 4 * s4 + q;
      r = r < nrows ? r : nrows - 1;
#pragma unroll
      for (int it = 0; it < NT; ++it) za[s4][it] = Z[r * B + 16 * it + (lane & 15)];
    }
  };

  double gacc[GRAM ? NG : 1];
#pragma unroll
  for (int p = 0; p < (GRAM ? NG : 1); ++p) gacc[p] = 0.0;
  d4v gx[XG ? NT : 1][XG ? NT : 1];
#pragma unroll
  for (int it = 0; it < (XG ? NT : 1); ++it)
#pragma unroll
    for (int jt = 0; jt < (XG ? NT : 1); ++jt) gx[it][jt] = d4v{0.0, 0.0, 0.0, 0.0};

  d2v xa[1][NH], ya[1][kYPer];
  double za[XG ? 4 : 1][XG ? NT : 1];
  const bool by = MODE == 0 && beta != 0.0;  // the CholQR forms have beta = 0: no Y registers
  const int64_t blk_c = blk < nblk ? blk : nblk - 1;
  load_x(blk_c, xa);
  if (by) load_y(blk_c, ya);
  if constexpr (XG) load_z(blk_c, za);
  for (; blk < nblk; blk += stride) {
    // keep the C operands in LDS: without this compiler barrier LLVM hoists their reads out
    // of the loop and holds 32 x 16 B per lane in registers (occupancy 1, spills)
    asm volatile("" ::: "memory");
    d2v xn[1][NH], yn[1][kYPer];
    double zn[XG ? 4 : 1][XG ? NT : 1];
    {
      const int64_t bn = blk + stride < nblk ? blk + stride : nblk - 1;  // clamped prefetch
      load_x(bn, xn);
      if (by) load_y(bn, yn);
      if constexpr (XG) load_z(bn, zn);
    }
    double acc[1][CG];
#pragma unroll
    for (int rt = 0; rt < 1; ++rt) {
      if (by) {  // beta Y into the D layout through the wave's LDS tile
#pragma unroll
        for (int m = 0; m < kYPer; ++m) {
          const int e = 2 * lane + 128 * m;
          *reinterpret_cast<d2v*>(ot + swz(e / B, e % B)) = beta * ya[rt][m];
        }
#pragma unroll
        for (int cg = 0; cg < CG; ++cg) acc[rt][cg] = ot[swz(4 * g + q, 4 * cg + j)];
      } else {
#pragma unroll
        for (int cg = 0; cg < CG; ++cg) acc[rt][cg] = 0.0;
      }
      // acc += X (alpha C): k = 8h + 2q + v
#pragma unroll
      for (int h = 0; h < NH; ++h)
#pragma unroll
        for (int v = 0; v < 2; ++v) {
          const double a = v ? xa[rt][h].y : xa[rt][h].x;
          const double* cb = cs + (8 * h + 2 * q + v) * LDC + 2 * j;
          mfma_row<TRI>(8 * h + v, a, cb, acc[rt]);
        }
      if constexpr (TWO) {
        // Q1 tile (D layout) -> the wave's LDS stage -> A layout; acc = Q1 C2, the same MFMA
        // order as a separate apply pass reading Q1 back from HBM (bit-identical)
#pragma unroll
        for (int cg = 0; cg < CG; ++cg) ot[swz(4 * g + q, 4 * cg + j)] = acc[rt][cg];
        d2v x2[NH];
#pragma unroll
        for (int h = 0; h < NH; ++h) x2[h] = *reinterpret_cast<const d2v*>(ot + swz(lane & 15, 8 * h + 2 * q));
#pragma unroll
        for (int cg = 0; cg < CG; ++cg) acc[rt][cg] = 0.0;
#pragma unroll
        for (int h = 0; h < NH; ++h)
#pragma unroll
          for (int v = 0; v < 2; ++v) {
            const double a = v ? x2[h].y : x2[h].x;
            const double* cb = cs2 + (8 * h + 2 * q + v) * LDC + 2 * j;
            mfma_row<TRI>(8 * h + v, a, cb, acc[rt]);
          }
      }
      const int64_t rbase = blk * kBlockRows + 16 * rt;
      if constexpr (GRAM) {
        // rows past the end (clamped loads) must not enter the Gram
        const bool live = rbase + 4 * g + q < nrows;
        double am[CG];
#pragma unroll
        for (int cg = 0; cg < CG; ++cg) am[cg] = live ? acc[rt][cg] : 0.0;
        int p = 0;
#pragma unroll
        for (int ic = 0; ic < CG; ++ic)
#pragma unroll
          for (int jc = ic; jc < CG; ++jc, ++p) gacc[p] = mfma4r(am[ic], am[jc], gacc[p]);
      }
      // Y' out: D layout -> LDS -> row-major 16-B stores
      if constexpr (STORE || XG) {
#pragma unroll
        for (int cg = 0; cg < CG; ++cg) ot[swz(4 * g + q, 4 * cg + j)] = acc[rt][cg];
      }
      if constexpr (XG) {
        // Z^T Y' over the tile's live rows (Z rows past the end read as 0)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          const bool lz = rbase + 4 * s4 + q < nrows;
#pragma unroll
          for (int jt = 0; jt < NT; ++jt) {
            const double yb = ot[swz(4 * s4 + q, 16 * jt + (lane & 15))];
#pragma unroll
            for (int it = 0; it < NT; ++it)
              gx[it][jt] = __builtin_amdgcn_mfma_f64_16x16x4f64(lz ? za[s4][it] : 0.0, yb, gx[it][jt], 0, 0, 0);
          }
        }
      }
#pragma unroll
      for (int m = 0; m < (STORE ? kYPer : 0); ++m) {
        const int e = 2 * lane + 128 * m;
        const int64_t r = rbase + e / B;
        const d2v v = *reinterpret_cast<const d2v*>(ot + swz(e / B, e % B));
        if (r < nrows) {
          if (w64) stnt(v, reinterpret_cast<d2v*>(Y + r * B + (e % B)));
          else *reinterpret_cast<float2*>(Y32 + r * B + (e % B)) = make_float2((float)v.x, (float)v.y);
        }
      }
    }
#pragma unroll
    for (int rt = 0; rt < 1; ++rt) {
#pragma unroll
      for (int h = 0; h < NH; ++h) xa[rt][h] = xn[rt][h];
#pragma unroll
      for (int m = 0; m < kYPer; ++m) ya[rt][m] = yn[rt][m];
    }
    if constexpr (XG) {
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int it = 0; it < NT; ++it) za[s4][it] = zn[s4][it];
    }
  }
  if constexpr (GRAM) {
    // sum the four row-quad blocks (lane bits 2, 3), then the four waves, into slab[block]
    __syncthreads();  // the LDS is reused
    double* gw = gs + wave * B * B;
    int p = 0;
#pragma unroll
    for (int ic = 0; ic < CG; ++ic)
#pragma unroll
      for (int jc = ic; jc < CG; ++jc, ++p) {
        double v = gacc[p];
        v += __shfl_xor(v, 4, 64);
        v += __shfl_xor(v, 8, 64);
        if (g == 0) {
          const int r = 4 * ic + q, c = 4 * jc + j;
          gw[r * B + c] = v;
          if (ic != jc) gw[c * B + r] = v;  // lower triangle of the off-diagonal quads
        }
      }
    __syncthreads();
    double* out = slab + (int64_t)blockIdx.x * B * B;
    for (int e = tid; e < B * B; e += kRowThreads)
      out[e] = (gs[e] + gs[B * B + e]) + (gs[2 * B * B + e] + gs[3 * B * B + e]);
  }
  if constexpr (XG) {
    // 16x16x4 D layout: gx[it][jt][reg] = (Z^T Y')[16 it + q + 4 reg][16 jt + (lane & 15)]
    __syncthreads();
    double* gw = gs + wave * B * B;
#pragma unroll
    for (int it = 0; it < NT; ++it)
#pragma unroll
      for (int jt = 0; jt < NT; ++jt)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg)
          gw[(16 * it + q + 4 * reg) * B + 16 * jt + (lane & 15)] = gx[it][jt][reg];
    __syncthreads();
    double* out = slab2 + (int64_t)blockIdx.x * B * B;
    for (int e = tid; e < B * B; e += kRowThreads)
      out[e] = (gs[e] + gs[B * B + e]) + (gs[2 * B * B + e] + gs[3 * B * B + e]);
  }
}

// workgroups per CU the instantiation holds (its VGPRs), cached; the persistent grid is this
// many per CU, capped at kMaxPerCu, so every workgroup is resident from the start
constexpr int kMaxPerCu = 4;
template <int B, bool GRAM, bool XF, bool YF, int MODE, bool XG, bool TRI>
int rg_per_cu() {
  static std::atomic<int> per{0};
  int v = per.load(std::memory_order_relaxed);
  if (v == 0) {
    int nb = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&nb, k_rowgram<B, GRAM, XF, YF, MODE, XG, TRI>,
                                                     kRowThreads, 0) != hipSuccess || nb < 1)
      nb = 2;
    v = nb < kMaxPerCu ? nb : kMaxPerCu;
    per.store(v, std::memory_order_relaxed);
  }
  return v;
}

template <int B, bool GRAM, bool XF, bool YF, int MODE, bool XG, bool TRI>
void launch_rg_t(const RowOpArgs& a, int64_t nrows, int grid, hipStream_t s) {
  if (grid <= 0) grid = rowgram_grid(nrows, rg_per_cu<B, GRAM, XF, YF, MODE, XG, TRI>());
  if (a.grid_out) *a.grid_out = grid;
  hipLaunchKernelGGL((k_rowgram<B, GRAM, XF, YF, MODE, XG, TRI>), dim3(grid), dim3(kRowThreads), 0, s,
                     nrows, a.X, a.C, a.ldc, a.Y, a.alpha, a.beta, a.slab, a.skip, a.X32, a.Y32,
                     a.f64flag, a.C2, a.Z, a.slab2);
}
// the triangular form for the fp64-X instantiations (CholQR's applies); fp32-X stays general
template <int B, bool GRAM, bool XF, bool YF, int MODE, bool XG>
void launch_rg(const RowOpArgs& a, int64_t nrows, int grid, hipStream_t s) {
  if constexpr (!XF) {
    if (a.tri) return launch_rg_t<B, GRAM, XF, YF, MODE, XG, true>(a, nrows, grid, s);
  }
  launch_rg_t<B, GRAM, XF, YF, MODE, XG, false>(a, nrows, grid, s);
}

template <int B>
bool launch_rowgram(const RowOpArgs& a, int64_t nrows, int grid, hipStream_t s) {
  const bool gram = a.slab != nullptr, xg = a.Z != nullptr;
  if (a.mode == 0 && !xg) {
    if (a.X32 && a.Y32) {
      if (gram) launch_rg<B, true, true, true, 0, false>(a, nrows, grid, s);
      else launch_rg<B, false, true, true, 0, false>(a, nrows, grid, s);
    } else if (a.X32) {
      if (gram) launch_rg<B, true, true, false, 0, false>(a, nrows, grid, s);
      else launch_rg<B, false, true, false, 0, false>(a, nrows, grid, s);
    } else if (a.Y32) {
      if (gram) launch_rg<B, true, false, true, 0, false>(a, nrows, grid, s);
      else launch_rg<B, false, false, true, 0, false>(a, nrows, grid, s);
    } else {
      if (gram) launch_rg<B, true, false, false, 0, false>(a, nrows, grid, s);
      else launch_rg<B, false, false, false, 0, false>(a, nrows, grid, s);
    }
    return true;
  }
  if (a.X32) return false;
  if (a.mode == 0 && xg && !gram) {  // CholQR pass 3 with the next step's local-reorth Gram
    if (a.Y32) launch_rg<B, false, false, true, 0, true>(a, nrows, grid, s);
    else launch_rg<B, false, false, false, 0, true>(a, nrows, grid, s);
    return true;
  }
  if (a.mode == 1 && gram && !xg && !a.Y32) {
    launch_rg<B, true, false, false, 1, false>(a, nrows, grid, s);
    return true;
  }
  if (a.mode == 2 && !gram) {  // (the pass-3 Gram, when a shifted pass 1 asks for it, is a
                               // separate skip-flagged pass: it would spill here beside XG)
    if (xg) {
      if (a.Y32) launch_rg<B, false, false, true, 2, true>(a, nrows, grid, s);
      else launch_rg<B, false, false, false, 2, true>(a, nrows, grid, s);
    } else {
      if (a.Y32) launch_rg<B, false, false, true, 2, false>(a, nrows, grid, s);
      else launch_rg<B, false, false, false, 2, false>(a, nrows, grid, s);
    }
    return true;
  }
  return false;
}

}  // namespace

bool rowgram_ok(int b) { return b == 16 || b == 32; }

int rowgram_grid(int64_t nrows, int per_cu) {
  // per_cu workgroups per CU (two at b = 32 with the Gram: register-bound); never more
  // blocks than rows need
  int64_t g = (int64_t)per_cu * window_grid();
  const int64_t need = (nrows + 4 * kBlockRows - 1) / (4 * kBlockRows);
  if (g > need) g = need;
  return (int)(g < 1 ? 1 : g);
}

bool rowgram_ex(int64_t nrows, int b, const RowOpArgs& a, int grid, hipStream_t s) {
  if (b == 32) return launch_rowgram<32>(a, nrows, grid, s);
  if (b == 16) return launch_rowgram<16>(a, nrows, grid, s);
  return false;
}

void rowgram(int64_t nrows, int b, const double* X, const double* C, int ldc, double* Y,
             double alpha, double beta, double* slab, int grid, const int* skip, hipStream_t s,
             const float* X32, float* Y32, const int* f64flag, bool tri) {
  RowOpArgs a;
  a.tri = tri;
  a.X = X;
  a.C = C;
  a.ldc = ldc;
  a.Y = Y;
  a.alpha = alpha;
  a.beta = beta;
  a.slab = slab;
  a.skip = skip;
  a.X32 = X32;
  a.Y32 = Y32;
  a.f64flag = f64flag;
  rowgram_ex(nrows, b, a, grid, s);
}

}  // namespace rbl
