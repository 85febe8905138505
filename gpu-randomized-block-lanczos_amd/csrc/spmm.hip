// spmm.hip — CSR block SpMM  U = A * Q_i  (+ fused 3-term epilogue  U -= Q_{i-1} B_i^T).
//
// Replaces cuSPARSE SpMM `mul!(U, Ag, Qg_d)` (RBL_gpu.jl:152,176,214) and the following
// cuBLAS gemm `mul!(U, Qg1_d, transpose(Big), -1, 1)` (RBL_gpu.jl:177).  A is symmetric, so
// the CSC arrays the reference uploads are the CSR arrays used here.
//
// Q blocks are row-major n x b: the gather of Q[c,:] is one contiguous b*8-byte segment.
// Memory-bound: algorithmic bytes nnz*(8+4) + (n+1)*8 + 2*n*b*8 per call.
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
                                                     const double* __restrict__ Bi) {
  constexpr int G = kWave / BP;
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= nrows) return;
  const int g = lane / BP, c = lane % BP;
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

template <int BP>
static void launch_gather(const CsrDev& A, const double* Q, int64_t off, int b, double* U,
                          const double* Qprev, const double* Bi, hipStream_t s) {
  const int64_t blocks = (A.nrows + 3) / 4;
  hipLaunchKernelGGL((k_spmm_gather<BP>), dim3((unsigned)blocks), dim3(256), 0, s, A.nrows,
                     A.rowptr, A.col, A.val, Q, off, b, U, Qprev, Bi);
}

int spmm(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
         const double* Qprev, const double* Bi, int variant, hipStream_t s, double* ai_slab) {
  if (A.nrows <= 0) return 0;
  // 0 auto: band tiles > band (MFMA) > window (DPP) > gather;  1 gather;  2 window;  3 band;
  // 4 band tiles
  int parts = 0;
  if ((variant == 0 || variant == 4) &&
      spmm_bt(A, Qin, col_off, b, U, Qprev, Bi, s, ai_slab, &parts))
    return parts;
  if ((variant == 0 || variant == 3 || variant == 4) &&
      spmm_band(A, Qin, col_off, b, U, Qprev, Bi, s, ai_slab, &parts))
    return parts;
  if ((variant == 0 || variant == 2 || variant == 3) &&
      spmm_window(A, Qin, col_off, b, U, Qprev, Bi, s))
    return 0;
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
