// spmm_band.hip — persistent CSR SpMM for banded sparsity with the band tile densified in
// LDS and multiplied on fp64 MFMA (gfx950).
//
// U = A * Q_i (+ fused 3-term epilogue U -= Q_{i-1} B_i^T) — RBL_gpu.jl:176-177.
// HBM traffic is exactly the CSR stream (nnz*(8+4) + (n+1)*8) plus Q_i, Q_{i-1} and U once.
//
// Why: a row-per-nonzero kernel (spmm_window.hip) reads one b*8-byte Q row from LDS per
// nonzero; at n=1e7, nnz=1e9, b=32 that is 256 GB of LDS reads — ~2.7 ms at the measured
// ds_read_b128 ceiling, as long as the whole HBM stream.  Here each 16-row tile's band
// (columns [cmin, cmax], <= 160 wide) is scattered from CSR into a dense LDS tile and
// multiplied with the Q ring rows by v_mfma_f64_4x4x4f64: every Q ring row is read once per
// tile (not once per nonzero), ~9 LDS reads per 8 MFMAs.  The zero fill costs flops
// (16 x K dense vs nnz), which the MFMA pipe absorbs while HBM stays the bound.
//
// Workgroup: 1024 threads (16 waves), one per CU, persistent over a contiguous tile range.
//   * staging (two tiles ahead, as spmm_window.hip): wave w loads row 16T+w's CSR entries
//     (coalesced), the tile's new ring rows, its Q_{i-1} rows and the descriptor of tile T+2
//     into registers; after the intervening tile computes, wave w zeroes its dense row and
//     scatters its entries (same wave, LDS writes in order: no barrier between the two).
//   * compute: wave w owns column group cg = w % (b/4) and k-split h = w / (b/4); it runs
//     its share of the tile's k-steps (and of the epilogue's b/4 k-steps against B_i^T held
//     in registers) into one fp64 accumulator per lane; k-split partials meet in LDS after
//     the tile barrier and the h = 0 wave stores the 16 x 4 block of U.
// v_mfma_f64_4x4x4f64 layout (tools/mfma_layout_probe.hip), block g = (lane>>2)&3 on row
// quad g: A[row = lane&15][k = lane>>4], B[k = lane>>4][col = lane&3], D[row 4g + (lane>>4)][lane&3].
#include <cstdlib>
#include <type_traits>

#include "kernels.hpp"

namespace rbl {

namespace band {
constexpr int kTileRows = 16;
constexpr int kThreads = 1024;
constexpr int kMaxK = 160;            // band width per tile (columns)
// dense tile rows: columns stored at perm8(k) so a lane's k-steps u, u+1 (columns k, k+4)
// come in one ds_read_b128; the 16 rows of a lane group land on distinct 16-B bank slots
// when kAdLd = 4 mod 32 (slot(r, q) = 2r + q mod 16 over each group's (r, q) set)
constexpr int kAdLd = kMaxK + 4;
constexpr int kRing = 256;            // ring rows
}  // namespace band

__device__ __forceinline__ double mfma4b(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

struct BandArgs {
  int64_t nrows;
  int64_t nnz;
  int64_t ntiles;
  int64_t tiles_per_wg;
  const int64_t* rowptr;
  const int32_t* col;
  const double* val;
  const int64_t* tinfo;  // per tile: e0, nnz, lo, hi, cmin, cmax, 0, 0
  const double* Q;
  int64_t col_off;
  double* U;
  const double* Qprev;
  const double* Bi;
  int ablate;  // diagnostics only (RBL_SPMM_ABLATE): 1 skip compute, 2 skip CSR/Q loads
};

template <int B>
struct BandLayout {
  static constexpr int NCG = B / 4;            // column groups of 4
  static constexpr int KSPLIT = 16 / NCG;      // waves per column group
  static constexpr int RLD = B + (B == 32 ? 4 : 4);  // ring row stride (doubles): 36 / 20
  static constexpr int QPLD = 36;              // Q_{i-1} tile stride, = 4 mod 32 (as kAdLd)
  static constexpr int kRingOff = 0;
  static constexpr int kRingBytes = band::kRing * RLD * 8;
  static constexpr int kAdOff = kRingBytes;
  static constexpr int kAdBytes = band::kTileRows * band::kAdLd * 8;
  static constexpr int kQpOff = kAdOff + 2 * kAdBytes;
  static constexpr int kQpBytes = band::kTileRows * QPLD * 8;
  static constexpr int kXchOff = kQpOff + 2 * kQpBytes;
  static constexpr int kXchBytes = (KSPLIT - 1) * NCG * 64 * 8;
  static constexpr int kDescOff = kXchOff + 2 * kXchBytes;
  static constexpr int kLds = kDescOff + 2 * 16;
};

struct BandStage {
  int c[3];
  double v[3];
  double q;
  double qp;
  int64_t desc_next;  // lane l <= 16: rowptr[16T'+l]; 17..20: lo, hi, cmin, cmax of T'
  int64_t rs, re, lo, hi, cmin, cmax;  // of the tile this stage holds (wave-uniform)
};

__device__ __forceinline__ int64_t bfield(int64_t v, int f) {
  const int lo = __builtin_amdgcn_readlane((int)(v & 0xffffffffll), f);
  const int hi = __builtin_amdgcn_readlane((int)(v >> 32), f);
  return ((int64_t)hi << 32) | (unsigned)lo;
}

template <int B, bool EPI>
__global__ __launch_bounds__(band::kThreads) void k_spmm_band(BandArgs a) {
  using L = BandLayout<B>;
  constexpr int NCG = L::NCG, KSPLIT = L::KSPLIT, RLD = L::RLD, QPLD = L::QPLD;
  constexpr int EKS = (B / 4) / KSPLIT;  // epilogue k-steps per wave
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* ring = reinterpret_cast<double*>(smem + L::kRingOff);
  auto adb = [&](int buf) { return reinterpret_cast<double*>(smem + L::kAdOff + buf * L::kAdBytes); };
  auto qpb = [&](int buf) { return reinterpret_cast<double*>(smem + L::kQpOff + buf * L::kQpBytes); };
  auto xcb = [&](int buf) { return reinterpret_cast<double*>(smem + L::kXchOff + buf * L::kXchBytes); };
  auto dsb = [&](int buf) { return reinterpret_cast<int*>(smem + L::kDescOff + buf * 16); };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = wave % NCG, h = wave / NCG;
  const int64_t t0 = (int64_t)blockIdx.x * a.tiles_per_wg;
  const int64_t t1 = t0 + a.tiles_per_wg < a.ntiles ? t0 + a.tiles_per_wg : a.ntiles;
  if (t0 >= t1) return;

  // every prefetch load below is unconditional (clamped address, masked at the LDS store):
  // each stage issues a fixed number of VMEM ops, so the compiler's vmcnt waits count only
  // the stage being consumed instead of draining the whole pipeline (vmcnt(0))
  auto load_desc = [&](int64_t t) -> int64_t {
    const int64_t tc = t < t1 ? t : t1 - 1;
    const int64_t r = tc * band::kTileRows + lane;
    const int64_t* p = lane <= 16 ? a.rowptr + (r < a.nrows ? r : a.nrows)
                                  : a.tinfo + tc * 8 + 2 + (lane <= 20 ? lane - 17 : 0);
    return *p;
  };
  auto load_stage = [&](int64_t t, BandStage& S) {
    S.rs = bfield(S.desc_next, wave);
    S.re = bfield(S.desc_next, wave + 1);
    S.lo = bfield(S.desc_next, 17);
    S.hi = bfield(S.desc_next, 18);
    S.cmin = bfield(S.desc_next, 19);
    S.cmax = bfield(S.desc_next, 20);
    S.desc_next = load_desc(t + 2);
    const int64_t last = a.nnz - 1;
    if (a.ablate == 2) return;  // diagnostics: stale stage data, real descriptors
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int64_t e = S.rs + lane + 64 * j;
      const int64_t ec = e < last ? e : last;
      S.c[j] = a.col[ec];
      S.v[j] = a.val[ec];
    }
    const int64_t row = S.lo + tid / B;
    const int64_t rowc = row < S.hi ? row : S.cmin;  // S.cmin: a valid row of Qin
    S.q = a.Q[(rowc - a.col_off) * B + (tid % B)];
    if constexpr (EPI) {
      const int64_t pr = t * band::kTileRows + (tid / B);
      S.qp = a.Qprev[(pr < a.nrows ? pr : a.nrows - 1) * B + (tid % B)];
    }
  };
  auto store_stage = [&](int64_t t, const BandStage& S) {
    if (t >= t1) return;
    const int buf = (int)(t & 1);
    double* ad = adb(buf) + wave * band::kAdLd;
    // wave w owns dense row w: zero it, then scatter (in-order LDS writes of one wave)
    for (int k = lane; k < band::kAdLd; k += 64) ad[k] = 0.0;
    const int cmin = (int)S.cmin;
#pragma unroll
    for (int j = 0; j < 3; ++j) {
      const int64_t e = S.rs + lane + 64 * j;
      if (e < S.re) ad[perm8(S.c[j] - cmin)] = S.v[j];
    }
    const int64_t row = S.lo + tid / B;
    if (row < S.hi) ring[(row & (band::kRing - 1)) * RLD + (tid % B)] = S.q;
    if constexpr (EPI) {
      if (tid < band::kTileRows * B) qpb(buf)[(tid / B) * QPLD + perm8(tid % B)] = S.qp;
    }
    if (tid == 0) {
      dsb(buf)[0] = cmin;
      dsb(buf)[1] = (int)(S.cmax - S.cmin + 1);
    }
  };

  // epilogue operand: B_i^T[k][c] = B_i[c][k] for this wave's column group and k-steps
  double bt[EPI ? EKS : 1];
  if constexpr (EPI) {
#pragma unroll
    for (int e = 0; e < EKS; ++e) {
      const int k = 4 * (h * EKS + e) + (lane >> 4);
      bt[e] = -a.Bi[(4 * cg + (lane & 3)) * B + k];
    }
  }

  double pend = 0.0;  // h == 0: accumulator of the tile awaiting its k-split partners
  auto compute = [&](int64_t t) {
    if (a.ablate == 1) return;  // diagnostics: pipeline only
    const int buf = (int)(t & 1);
    const int cmin = dsb(buf)[0], K = dsb(buf)[1];
    const int ks = (K + 3) >> 2;
    const int half = ((ks + 2 * KSPLIT - 1) / (2 * KSPLIT)) * 2;  // even: k-step pairs align
    const int kb = h * half;
    const int ke = kb + half < ks ? kb + half : ks;
    // lane (row r, q): column 4 k' + q sits at perm8(4 k' + q) = 8 (k'/2) + 2q + (k'&1)
    const double* ad = adb(buf) + (lane & 15) * band::kAdLd + 2 * (lane >> 4);
    const int bcol = 4 * cg + (lane & 3);
    double acc = 0.0;
    int kk = kb;
    for (; kk + 4 <= ke; kk += 4) {  // 4 k-steps: 2 x 16-B A reads + 4 B reads, 4 MFMAs
      d2v av[2];
      double bv[4];
#pragma unroll
      for (int u = 0; u < 2; ++u) av[u] = *reinterpret_cast<const d2v*>(ad + 8 * ((kk >> 1) + u));
#pragma unroll
      for (int u = 0; u < 4; ++u)
        bv[u] = ring[((cmin + 4 * (kk + u) + (lane >> 4)) & (band::kRing - 1)) * RLD + bcol];
      acc = mfma4b(av[0].x, bv[0], acc);
      acc = mfma4b(av[0].y, bv[1], acc);
      acc = mfma4b(av[1].x, bv[2], acc);
      acc = mfma4b(av[1].y, bv[3], acc);
    }
    for (; kk < ke; ++kk) {
      const int k = 4 * kk;
      acc = mfma4b(ad[perm8(k)], ring[((cmin + k + (lane >> 4)) & (band::kRing - 1)) * RLD + bcol], acc);
    }
    if constexpr (EPI) {
      const double* qp = qpb(buf) + (lane & 15) * QPLD + 2 * (lane >> 4);
      if constexpr (EKS % 2 == 0) {
#pragma unroll
        for (int e = 0; e < EKS; e += 2) {
          const d2v qv = *reinterpret_cast<const d2v*>(qp + 8 * ((h * EKS + e) >> 1));
          acc = mfma4b(qv.x, bt[e], acc);
          acc = mfma4b(qv.y, bt[e + 1], acc);
        }
      } else {
#pragma unroll
        for (int e = 0; e < EKS; ++e) acc = mfma4b(qp[perm8(4 * (h * EKS + e))], bt[e], acc);
      }
    }
    if (h > 0) {
      xcb(buf)[((h - 1) * NCG + cg) * 64 + lane] = acc;
    } else {
      pend = acc;
    }
  };
  auto finalize = [&](int64_t t) {
    if (h != 0) return;
    const int buf = (int)(t & 1);
    double acc = pend;
#pragma unroll
    for (int s = 1; s < KSPLIT; ++s) acc += xcb(buf)[((s - 1) * NCG + cg) * 64 + lane];
    const int g = (lane >> 2) & 3;
    const int64_t r = t * band::kTileRows + 4 * g + (lane >> 4);
    if (r < a.nrows) a.U[r * B + 4 * cg + (lane & 3)] = acc;
  };

  // ---- prologue ----
  // ring slots never loaded feed the zero padding columns (k >= K): make them finite zeros
  for (int i = tid; i < band::kRing * RLD; i += band::kThreads) ring[i] = 0.0;
  __syncthreads();
  {
    BandStage S0;
    S0.desc_next = load_desc(t0);
    const int64_t lo = bfield(S0.desc_next, 19), hi = bfield(S0.desc_next, 20) + 1;
    for (int64_t e = tid; e < (hi - lo) * B; e += band::kThreads) {
      const int64_t row = lo + e / B;
      ring[(row & (band::kRing - 1)) * RLD + (e % B)] = a.Q[(row - a.col_off) * B + (e % B)];
    }
    load_stage(t0, S0);
    store_stage(t0, S0);
    BandStage S1;
    S1.desc_next = load_desc(t0 + 1);
    load_stage(t0 + 1, S1);
    store_stage(t0 + 1, S1);
  }
  BandStage SA, SB;
  SA.desc_next = load_desc(t0 + 2);
  SB.desc_next = load_desc(t0 + 3);
  load_stage(t0 + 2, SA);
  load_stage(t0 + 3, SB);
  __syncthreads();

  for (int64_t t = t0; t < t1; t += 2) {
    compute(t);
    __syncthreads();
    finalize(t);
    store_stage(t + 2, SA);
    load_stage(t + 4, SA);
    if (t + 1 < t1) {
      compute(t + 1);
      __syncthreads();
      finalize(t + 1);
      store_stage(t + 3, SB);
      load_stage(t + 5, SB);
    }
  }
}

template <int B, bool EPI>
static void launch_band_t(const BandArgs& a, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_spmm_band<B, EPI>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, BandLayout<B>::kLds);
    attr = true;
  }
  hipLaunchKernelGGL((k_spmm_band<B, EPI>), dim3(grid), dim3(band::kThreads), BandLayout<B>::kLds,
                     s, a);
}

bool spmm_band(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
               const double* Qprev, const double* Bi, hipStream_t s) {
  if (A.ntiles <= 0 || !((b == 16 && A.band_ok16) || (b == 32 && A.band_ok32))) return false;
  BandArgs a;
  a.nrows = A.nrows;
  a.nnz = A.nnz;
  a.ntiles = A.ntiles;
  a.tiles_per_wg = A.tiles_per_wg;
  a.rowptr = A.rowptr;
  a.col = A.col;
  a.val = A.val;
  a.tinfo = A.tile_info;
  a.Q = Qin;
  a.col_off = col_off;
  a.U = U;
  a.Qprev = Qprev;
  a.Bi = Bi;
  static const int ablate = [] {
    const char* e = getenv("RBL_SPMM_ABLATE");
    return e ? atoi(e) : 0;
  }();
  a.ablate = ablate;
  const int grid = (int)((A.ntiles + A.tiles_per_wg - 1) / A.tiles_per_wg);
  const bool epi = Qprev != nullptr;
  if (b == 32) {
    if (epi) launch_band_t<32, true>(a, grid, s); else launch_band_t<32, false>(a, grid, s);
  } else {
    if (epi) launch_band_t<16, true>(a, grid, s); else launch_band_t<16, false>(a, grid, s);
  }
  return true;
}

}  // namespace rbl
