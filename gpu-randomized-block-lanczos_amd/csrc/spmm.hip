// spmm.hip — CSR block SpMM  U = A * Q_i  (+ fused 3-term epilogue  U -= Q_{i-1} B_i^T).
//
// Replaces cuSPARSE SpMM `mul!(U, Ag, Qg_d)` (RBL_gpu.jl:152,176,214) and the following
// cuBLAS gemm `mul!(U, Qg1_d, transpose(Big), -1, 1)` (RBL_gpu.jl:177).  A is symmetric, so
// the CSC arrays the reference uploads are the CSR arrays used here.
//
// Q blocks are row-major n x b: the gather of Q[c,:] is one contiguous b*8-byte segment.
// Memory-bound: algorithmic bytes nnz*(8+4) + (n+1)*8 + 2*n*b*8 per call.
#include <algorithm>
#include <cstdlib>

#include "kernels.hpp"

namespace rbl {

// ----------------------------------------------------------------------------------------
// Variant 1 — global gather.  One wave per row; the wave is split into G = 64/BP lane
// groups, group g takes nonzeros g, g+G, ...; lane c of a group owns column c of the row.
// Works for any sparsity pattern (R-MAT etc.); Q rows are served by L2 / Infinity Cache.
// ----------------------------------------------------------------------------------------
template <int BP>
__global__ __launch_bounds__(256) void k_spmm_gather(int64_t nrows, const int64_t* __restrict__ rowptr,
                                                     const int32_t* __restrict__ col,
                                                     const double* __restrict__ val,
                                                     const double* __restrict__ Q, int64_t col_off,
                                                     int b, double* __restrict__ U,
                                                     const double* __restrict__ Qprev,
                                                     const double* __restrict__ Bi, int ncb) {
  constexpr int G = kWave / BP;
  const int lane = threadIdx.x & 63;
  // b > 64: ncb waves per row, wave cb owning columns [64 cb, 64 cb + 64)
  const int64_t wid = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int64_t row = wid / ncb;
  if (row >= nrows) return;
  const int g = lane / BP, c = (int)(wid % ncb) * BP + lane % BP;
  const bool cv = c < b;
  const int cs = cv ? c : 0;
  const int64_t s = rowptr[row], e = rowptr[row + 1];
  double acc0 = 0.0, acc1 = 0.0;
  int64_t k = s + g;
  for (; k + 3 * G < e; k += 4 * G) {
    const int64_t c0 = col[k] - col_off, c1 = col[k + G] - col_off;
    const int64_t c2 = col[k + 2 * G] - col_off, c3 = col[k + 3 * G] - col_off;
    const double v0 = val[k], v1 = val[k + G], v2 = val[k + 2 * G], v3 = val[k + 3 * G];
    const double q0 = Q[c0 * b + cs], q1 = Q[c1 * b + cs];
    const double q2 = Q[c2 * b + cs], q3 = Q[c3 * b + cs];
    acc0 = fma(v0, q0, acc0);
    acc1 = fma(v1, q1, acc1);
    acc0 = fma(v2, q2, acc0);
    acc1 = fma(v3, q3, acc1);
  }
  for (; k < e; k += G) acc0 = fma(val[k], Q[(col[k] - col_off) * b + cs], acc0);
  double acc = acc0 + acc1;
#pragma unroll
  for (int m = BP; m < kWave; m <<= 1) acc += __shfl_xor(acc, m, kWave);
  if (g == 0 && cv) {
    if (Qprev) {
      const double* qp = Qprev + row * b;
      const double* bp = Bi + (int64_t)c * b;
      for (int t = 0; t < b; ++t) acc = fma(-qp[t], bp[t], acc);
    }
    U[row * b + c] = acc;
  }
}

// ----------------------------------------------------------------------------------------
// Variant 5 — segmented gather for unstructured power-law patterns (R-MAT),
// b in {16, 32}.  A per-matrix task table (CsrDev::seg_*) packs short rows into wave tasks of
// <= kSegPack nonzeros and cuts every row longer than kSegLen nonzeros into segments of its
// own tasks, so one hub row (R-MAT's vertex 0 has ~1e6 neighbours at C4b) no longer holds a
// single wave for the whole launch.  A lane group of BP lanes (one per column) owns a row:
// lane c loads entry k + c of a BP-entry chunk (coalesced col/val), then the group walks the
// chunk 8 entries at a time, broadcasting each (col, val) by __shfl and issuing the 8 Q-row
// gathers back to back.  Segments write partial rows to `scratch`; k_seg_fixup sums each long
// row's segments in order (deterministic) and applies the 3-term epilogue there.
// ----------------------------------------------------------------------------------------
#ifndef RBL_SEG_BLDS
#define RBL_SEG_BLDS 1
#endif
#ifndef RBL_SEG_PF
#define RBL_SEG_PF 0
#endif
#ifndef RBL_SEG_G
#define RBL_SEG_G 8  // Q-row gathers issued back to back per lane group
#endif
// minimum waves per SIMD (0: the compiler's choice).  b = 32 with B_i in LDS: 79 VGPRs, 6 waves;
// forcing 8 (62 VGPRs, no spill) measured the same (37.2 vs 37.05 ms, r03_seg_blds8_ab.log)
#ifndef RBL_SEG_WPE
#define RBL_SEG_WPE 0
#endif
// b = 16: 94 VGPRs, 5 waves; 6 or 8 spill (28 / 58 VGPRs), and B_i in LDS measured slower
#ifndef RBL_SEG_WPE16
#define RBL_SEG_WPE16 1
#endif
constexpr int kSegG = RBL_SEG_G;
#ifndef RBL_SEG_HOT
#define RBL_SEG_HOT 0
#endif
template <int BP>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(BP == 16 ? RBL_SEG_WPE16 : RBL_SEG_WPE ? RBL_SEG_WPE : 1))) void k_spmm_seg(
    int64_t ntasks, const int64_t* __restrict__ trow, const int32_t* __restrict__ tinfo,
    const int64_t* __restrict__ rowptr, const int32_t* __restrict__ col,
    const double* __restrict__ val, const double* __restrict__ Q, int64_t col_off,
    double* __restrict__ U, double* __restrict__ scratch, const int64_t* __restrict__ slot_k0,
    const double* __restrict__ Qprev, const double* __restrict__ Bi, bool accum) {
  constexpr int R = kWave / BP;
  const int lane = threadIdx.x & 63;
  const int64_t t = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  // BLDS (b = 32): B_i for the 3-term epilogue in LDS, bs[u * BP + c] = B_i[c][u] (a lane group
  // reads 256 consecutive bytes: conflict-free) instead of 32 doubles per lane in registers:
  // 126 -> 79 VGPRs, 4 -> 6 waves per SIMD, R-MAT SpMM 39.8 -> 37.5 ms, bit-identical
  // (profiles/r03_seg_blds_ab.log).  At b = 16 the register copy is 16 doubles and the LDS
  // reads cost more than the occupancy gains (C3 0.328 -> 0.335 ms), so it stays there.
  constexpr bool kBlds = RBL_SEG_BLDS && BP == 32;
  __shared__ double bs[kBlds ? BP * BP : 1];
  if constexpr (kBlds) {
    if (Qprev)
      for (int e = threadIdx.x; e < BP * BP; e += 256) bs[(e % BP) * BP + e / BP] = Bi[e];
    __syncthreads();
  }
  if (t >= ntasks) return;
  const int h = lane / BP, c = lane % BP;
  const int64_t r0 = trow[t];
  const int info = tinfo[t];
  // nonzeros [k, e) of one row, lane c: column c; chunks of BP entries, k stepping by `step`
  auto dot = [&](int64_t k, int64_t e, int64_t step) -> double {
    double acc0 = 0.0, acc1 = 0.0;
    // PF: the next chunk's col / val are loaded before this chunk's gathers issue, so their
    // latency hides behind the gathers instead of stalling the chunk's first round.  Measured
    // neutral at 5 and at 7 waves per SIMD (37.44 / 37.47 vs 37.43 ms, profiles/r03_seg_pf_ab.log):
    // the other waves already cover it.  Off.  A row pipeline over the lane group's rows (bounds
    // two rows ahead, first chunk one row ahead: the rowptr -> col -> Q chain of C3's ~5-nonzero
    // rows) measured the same at b = 16 (0.328 / 0.329 ms) and slower at b = 32 (37.8 vs 37.4 ms;
    // profiles/r03_seg_rowpipe_ab.log), so not kept.
    int cl_n = 0;
    double vl_n = 0.0;
    if constexpr (RBL_SEG_PF) {
      const int64_t kk = k + c;
      const bool ok = kk < e;
      cl_n = ok ? col[kk] : (int)col_off;
      vl_n = ok ? val[kk] : 0.0;
    }
    for (; k < e; k += step) {
      int cl;
      double vl;
      if constexpr (RBL_SEG_PF) {
        cl = cl_n;
        vl = vl_n;
        const int64_t kn = k + step + c;
        const bool okn = kn < e;
        cl_n = okn ? col[kn] : (int)col_off;
        vl_n = okn ? val[kn] : 0.0;
      } else {
        const int64_t kk = k + c;
        const bool ok = kk < e;
        cl = ok ? col[kk] : (int)col_off;  // padding: Q row 0 times 0
        vl = ok ? val[kk] : 0.0;
      }
      const int cnt = e - k < BP ? (int)(e - k) : BP;
      for (int j0 = 0; j0 < cnt; j0 += kSegG) {
        double q[kSegG], v[kSegG];
#pragma unroll
        for (int jj = 0; jj < kSegG; ++jj) {
          const int cj = __shfl(cl, j0 + jj, BP);
          v[jj] = __shfl(vl, j0 + jj, BP);
          const double* qp = Q + ((int64_t)(cj - col_off) * BP + c);
          if constexpr (RBL_SEG_HOT > 0) {
            // columns past the hot set (R-MAT: high ids, low degree) load non-temporally so the
            // hub rows' lines stay in L2 — measured no faster at hot sets of 16 K and 128 K
            // rows (profiles/r03_rmat_hot_nt_ab.log), so off
            if (cj < RBL_SEG_HOT) q[jj] = *qp;
            else q[jj] = __builtin_nontemporal_load(qp);
          } else {
            q[jj] = *qp;
          }
        }
#pragma unroll
        for (int jj = 0; jj < kSegG; jj += 2) {
          acc0 = fma(v[jj], q[jj], acc0);
          acc1 = fma(v[jj + 1], q[jj + 1], acc1);
        }
      }
    }
    return acc0 + acc1;
  };
  if (info > 0) {
    double bt[kBlds ? 1 : BP];  // epilogue operand B_i[c][t] (registers unless kBlds)
    if (!kBlds && Qprev) {
#pragma unroll
      for (int u = 0; u < (kBlds ? 1 : BP); ++u) bt[u] = Bi[c * BP + u];
    }
    for (int rr = h; rr < info; rr += R) {  // lane-group-uniform row loop
      const int64_t row = r0 + rr;
      double acc = dot(rowptr[row], rowptr[row + 1], BP);
      if (accum) acc += U[row * BP + c];  // a later column tier: add to the earlier sweeps
      if (Qprev) {
        const double qv = Qprev[row * BP + c];
#pragma unroll
        for (int u = 0; u < BP; ++u) {
          acc = fma(-__shfl(qv, u, BP), kBlds ? bs[u * BP + c] : bt[kBlds ? 0 : u], acc);
        }
      }
      U[row * BP + c] = acc;
    }
  } else {
    const int64_t slot = -(int64_t)info - 1;
    const int64_t k0 = slot_k0[slot], k1 = slot_k0[slot + 1];
    const int64_t e = rowptr[r0 + 1] < k1 ? rowptr[r0 + 1] : k1;
    double acc = dot(k0 + (int64_t)h * BP, e, (int64_t)R * BP);
#pragma unroll
    for (int m = BP; m < kWave; m <<= 1) acc += __shfl_xor(acc, m, kWave);
    if (h == 0) scratch[slot * BP + c] = acc;
  }
}

// long rows: the sum of their segments in slot order, then the 3-term epilogue
template <int BP>
__global__ __launch_bounds__(256) void k_seg_fixup(int64_t nlong, const int64_t* __restrict__ lrow,
                                                  const int64_t* __restrict__ lslot,
                                                  const double* __restrict__ scratch,
                                                  double* __restrict__ U,
                                                  const double* __restrict__ Qprev,
                                                  const double* __restrict__ Bi, bool accum) {
  constexpr int R = kWave / BP;
  const int lane = threadIdx.x & 63;
  const int64_t i = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / BP;
  (void)R;
  if (i >= nlong) return;
  const int c = lane % BP;
  const int64_t row = lrow[i];
  double acc = 0.0;
  for (int64_t sl = lslot[i]; sl < lslot[i + 1]; ++sl) acc += scratch[sl * BP + c];
  if (accum) acc += U[row * BP + c];
  if (Qprev) {
    for (int u = 0; u < BP; ++u) acc = fma(-Qprev[row * BP + u], Bi[c * BP + u], acc);
  }
  U[row * BP + c] = acc;
}

template <int BP>
static void launch_seg(const CsrDev::Tier& T, const double* Q, int64_t off, double* U,
                       const double* Qprev, const double* Bi, bool accum, hipStream_t s) {
  if (T.ntasks <= 0) return;
  const int64_t blocks = (T.ntasks + 3) / 4;
  hipLaunchKernelGGL((k_spmm_seg<BP>), dim3((unsigned)blocks), dim3(256), 0, s, T.ntasks,
                     T.trow, T.tinfo, T.rowptr, T.col, T.val, Q, off, U, T.scratch,
                     T.slot_k0, Qprev, Bi, accum);
  if (T.nlong > 0) {
    const int64_t th = T.nlong * BP;
    hipLaunchKernelGGL((k_seg_fixup<BP>), dim3((unsigned)((th + 255) / 256)), dim3(256), 0, s,
                       T.nlong, T.lrow, T.lslot, T.scratch, U, Qprev, Bi, accum);
  }
}

// the whole matrix as one tier, or (CsrDev::seg_ntiers) the column tiers in order: the first
// writes U, the others add to it, the last applies the 3-term epilogue
template <int BP>
static void launch_seg_all(const CsrDev& A, const double* Q, int64_t off, double* U,
                           const double* Qprev, const double* Bi, hipStream_t s) {
  if (A.seg_ntiers > 0) {
    for (int t = 0; t < A.seg_ntiers; ++t) {
      const bool last = t == A.seg_ntiers - 1;
      const double* Qt = Q;
      int64_t ot = off;
      if (A.seg_split && t == 0 && A.qloc) {  // own columns straight from the block
        Qt = static_cast<const double*>(A.qloc);
        ot = A.loc_lo;
      }
      if (A.seg_split && t == 1 && A.seg_wait) hipStreamWaitEvent(s, A.seg_wait, 0);
      launch_seg<BP>(A.seg_tier[t], Qt, ot, U, last ? Qprev : nullptr, Bi, t > 0, s);
    }
    return;
  }
  CsrDev::Tier T;
  T.rowptr = A.rowptr;
  T.col = A.col;
  T.val = A.val;
  T.ntasks = A.seg_ntasks;
  T.nlong = A.seg_nlong;
  T.trow = A.seg_trow;
  T.tinfo = A.seg_tinfo;
  T.slot_k0 = A.seg_slot_k0;
  T.lrow = A.seg_lrow;
  T.lslot = A.seg_lslot;
  T.scratch = A.seg_scratch;
  launch_seg<BP>(T, Q, off, U, Qprev, Bi, false, s);
}

// ---- column tiers: count, then fill (one thread per row; a one-off per matrix) ----
__global__ void k_seg_tier_count(int64_t m, const int64_t* __restrict__ rowptr,
                                 const int32_t* __restrict__ col, const uint8_t* __restrict__ tier_of,
                                 int ntiers, int32_t* __restrict__ cnt) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= m) return;
  int c3[kMaxSegTiers] = {0, 0, 0};
  for (int64_t k = rowptr[r]; k < rowptr[r + 1]; ++k) ++c3[tier_of[col[k]]];
  for (int t = 0; t < ntiers; ++t) cnt[t * m + r] = c3[t];
}

struct TierPtrs {
  int64_t* rp[kMaxSegTiers];
  int32_t* col[kMaxSegTiers];
  double* val[kMaxSegTiers];
};

__global__ void k_seg_tier_fill(int64_t m, const int64_t* __restrict__ rowptr,
                                const int32_t* __restrict__ col, const double* __restrict__ val,
                                const uint8_t* __restrict__ tier_of, TierPtrs tp) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= m) return;
  int64_t pos[kMaxSegTiers];
  for (int t = 0; t < kMaxSegTiers; ++t) pos[t] = tp.rp[t] ? tp.rp[t][r] : 0;
  for (int64_t k = rowptr[r]; k < rowptr[r + 1]; ++k) {
    const int c = col[k];
    const int t = tier_of[c];
    tp.col[t][pos[t]] = c;
    tp.val[t][pos[t]] = val[k];
    ++pos[t];
  }
}

void seg_tier_count(int64_t m, const int64_t* rowptr, const int32_t* col, const uint8_t* tier_of,
                    int ntiers, int32_t* cnt, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_seg_tier_count, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, m,
                     rowptr, col, tier_of, ntiers, cnt);
}

void seg_tier_fill(int64_t m, const int64_t* rowptr, const int32_t* col, const double* val,
                   const uint8_t* tier_of, int ntiers, int64_t* const* trp, int32_t* const* tcol,
                   double* const* tval, hipStream_t s) {
  if (m <= 0) return;
  TierPtrs tp;
  for (int t = 0; t < kMaxSegTiers; ++t) {
    tp.rp[t] = t < ntiers ? trp[t] : nullptr;
    tp.col[t] = t < ntiers ? tcol[t] : nullptr;
    tp.val[t] = t < ntiers ? tval[t] : nullptr;
  }
  hipLaunchKernelGGL(k_seg_tier_fill, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, m,
                     rowptr, col, val, tier_of, tp);
}

__device__ inline int tier_rule(const TierRule& R, int64_t r, int64_t c) {
  if (c >= R.r0 && c < R.r1) return 0;
  const int dc = R.deg[c], dr = R.deg[r];
  return (dc > dr || (dc == dr && c < r)) ? 1 : 2;
}
__global__ void k_seg_tier_count_rule(int64_t m, const int64_t* __restrict__ rowptr,
                                      const int32_t* __restrict__ col, TierRule R,
                                      int32_t* __restrict__ cnt) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= m) return;
  int c3[kMaxSegTiers] = {0, 0, 0};
  for (int64_t k = rowptr[r]; k < rowptr[r + 1]; ++k) ++c3[tier_rule(R, R.row0 + r, col[k])];
  for (int t = 0; t < kMaxSegTiers; ++t) cnt[t * m + r] = c3[t];
}
__global__ void k_seg_tier_fill_rule(int64_t m, const int64_t* __restrict__ rowptr,
                                     const int32_t* __restrict__ col, const double* __restrict__ val,
                                     TierRule R, TierPtrs tp) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= m) return;
  int64_t pos[kMaxSegTiers];
  for (int t = 0; t < kMaxSegTiers; ++t) pos[t] = tp.rp[t] ? tp.rp[t][r] : 0;
  for (int64_t k = rowptr[r]; k < rowptr[r + 1]; ++k) {
    const int c = col[k];
    const int t = tier_rule(R, R.row0 + r, c);
    tp.col[t][pos[t]] = c;
    tp.val[t][pos[t]] = val[k];
    ++pos[t];
  }
}
void seg_tier_count_rule(int64_t m, const int64_t* rowptr, const int32_t* col, TierRule rule,
                         int32_t* cnt, hipStream_t s) {
  if (m <= 0) return;
  hipLaunchKernelGGL(k_seg_tier_count_rule, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, m,
                     rowptr, col, rule, cnt);
}
void seg_tier_fill_rule(int64_t m, const int64_t* rowptr, const int32_t* col, const double* val,
                        TierRule rule, int64_t* const* trp, int32_t* const* tcol,
                        double* const* tval, hipStream_t s) {
  if (m <= 0) return;
  TierPtrs tp;
  for (int t = 0; t < kMaxSegTiers; ++t) {
    tp.rp[t] = trp[t];
    tp.col[t] = tcol[t];
    tp.val[t] = tval[t];
  }
  hipLaunchKernelGGL(k_seg_tier_fill_rule, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, m,
                     rowptr, col, val, rule, tp);
}

void spmm_seg_tier(const CsrDev::Tier& T, const double* Q, int64_t col_off, int b, double* out,
                   hipStream_t s) {
  if (b == 32) launch_seg<32>(T, Q, col_off, out, nullptr, nullptr, false, s);
  else launch_seg<16>(T, Q, col_off, out, nullptr, nullptr, false, s);
}

// one lane group (b lanes) per row with received partials; lane c sums column c in slot order
__global__ void k_push_add(const int64_t* __restrict__ rows, const int64_t* __restrict__ ptr,
                           const int64_t* __restrict__ slot, int64_t nrows,
                           const double* __restrict__ recv, int b, double* __restrict__ U) {
  const int64_t g = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / b;
  const int c = (int)(threadIdx.x % b);
  if (g >= nrows) return;
  double acc = 0.0;
  for (int64_t k = ptr[g]; k < ptr[g + 1]; ++k) acc += recv[slot[k] * b + c];
  U[rows[g] * b + c] += acc;
}
void push_add(const int64_t* rows, const int64_t* ptr, const int64_t* slot, int64_t nrows,
              const double* recv, int b, double* U, hipStream_t s) {
  if (nrows <= 0) return;
  const int64_t th = nrows * b;
  hipLaunchKernelGGL(k_push_add, dim3((unsigned)((th + 255) / 256)), dim3(256), 0, s, rows, ptr,
                     slot, nrows, recv, b, U);
}

bool spmm_seg_ok(const CsrDev& A, int b) { return A.seg_ntasks > 0 && (b == 16 || b == 32); }

template <int BP>
static void launch_gather(const CsrDev& A, const double* Q, int64_t off, int b, double* U,
                          const double* Qprev, const double* Bi, hipStream_t s) {
  const int ncb = (b + BP - 1) / BP;
  const int64_t blocks = (A.nrows * ncb + 3) / 4;
  hipLaunchKernelGGL((k_spmm_gather<BP>), dim3((unsigned)blocks), dim3(256), 0, s, A.nrows,
                     A.rowptr, A.col, A.val, Q, off, b, U, Qprev, Bi, ncb);
}

int spmm(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
         const double* Qprev, const double* Bi, int variant, hipStream_t s, double* ai_slab) {
  if (A.nrows <= 0) return 0;
  // 0 auto: band tiles > band (MFMA) > column panels > window (DPP) > segmented gather >
  // gather;  1 gather;  2 window;  3 band;  4 band tiles;  5 segmented gather;  7 column panels
  int parts = 0;
  if ((variant == 0 || variant == 4) &&
      spmm_bt(A, Qin, col_off, b, U, Qprev, Bi, s, ai_slab, &parts))
    return parts;
  // split sources: the band-tile kernel, or the own/halo column tiers of the segmented gather
  if (A.lfix_c) return -2;
  if (A.qloc && !(A.seg_split && (variant == 0 || variant == 5) && spmm_seg_ok(A, b))) return -2;
  if ((variant == 0 || variant == 3 || variant == 4) &&
      spmm_band(A, Qin, col_off, b, U, Qprev, Bi, s, ai_slab, &parts))
    return parts;
  if (((variant == 0 && A.panel_auto) || variant == 7) && spmm_panel(A, Qin, col_off, b, U, Qprev, Bi, s))
    return 0;
  if ((variant == 0 || variant == 2 || variant == 3) &&
      spmm_window(A, Qin, col_off, b, U, Qprev, Bi, s))
    return 0;
  if ((variant == 0 || variant == 5) && spmm_seg_ok(A, b)) {
    if (b == 32) launch_seg_all<32>(A, Qin, col_off, U, Qprev, Bi, s);
    else launch_seg_all<16>(A, Qin, col_off, U, Qprev, Bi, s);
    return 0;
  }
  if (b <= 1) launch_gather<1>(A, Qin, col_off, b, U, Qprev, Bi, s);
  else if (b <= 2) launch_gather<2>(A, Qin, col_off, b, U, Qprev, Bi, s);
  else if (b <= 4) launch_gather<4>(A, Qin, col_off, b, U, Qprev, Bi, s);
  else if (b <= 8) launch_gather<8>(A, Qin, col_off, b, U, Qprev, Bi, s);
  else if (b <= 16) launch_gather<16>(A, Qin, col_off, b, U, Qprev, Bi, s);
  else if (b <= 32) launch_gather<32>(A, Qin, col_off, b, U, Qprev, Bi, s);
  else launch_gather<64>(A, Qin, col_off, b, U, Qprev, Bi, s);
  return 0;
}

}  // namespace rbl
