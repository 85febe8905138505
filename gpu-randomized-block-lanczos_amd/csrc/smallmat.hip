// smallmat.hip — b x b work of the tall-skinny QR, on one workgroup, no host round trip.
//
// The reference factors every n x b block with cuSOLVER geqrf + orgqr (RBL_gpu.jl:155,
// 180-184; CPU: LAPACK, RBL.jl:102-104).  The HIP path uses CholQR2 and, when the block is
// (nearly) rank deficient — Krylov exhaustion in the reference's own tests —
// shifted CholQR3 (Fukaya et al. 2020: shift s = 11 (n b + b (b+1)) u ||U||^2, then two
// unshifted passes).  R has a non-negative diagonal.
#include <cstdlib>

#include "kernels.hpp"

namespace rbl {

constexpr int kMaxB = 64;  // b x b work in LDS up to here; larger b: global scratch (L2)

// M (the factor) and X (R^-1, then the Rtot product's scratch) live in LDS for b <= kMaxB and
// in a caller scratch of 2 b^2 doubles (L2-resident) above that: the block sizes past 64 that
// RBL_gpu(A, k, b) accepts (RBL_gpu.jl:205) take one more L2 trip per element, no LDS limit.
template <bool LDS>
struct SmallMat {
  double* p;
  int ld;
  __device__ double& operator()(int r, int c) const { return p[r * ld + c]; }
};

template <bool LDS>
__global__ __launch_bounds__(256) void k_chol(const double* __restrict__ G, int b, int64_t nglob,
                                              int mode, double* R, double* Rinv, double* Rtot,
                                              int* need3, int* status, const int* skip,
                                              double* scratch) {
  if (skip && *skip) return;
  __shared__ double Ml[LDS ? kMaxB * (kMaxB + 1) : 1];
  __shared__ double Xl[LDS ? kMaxB * (kMaxB + 1) : 1];
  __shared__ int fail;
  __shared__ double shift;
  __shared__ int zero;
  __shared__ double Gd[LDS ? kMaxB : 1];  // diag(G): the serial pivot / trace reads hit LDS, not L2
  const SmallMat<LDS> M{LDS ? Ml : scratch, LDS ? kMaxB + 1 : b};
  const SmallMat<LDS> X{LDS ? Xl : scratch + (int64_t)b * b, LDS ? kMaxB + 1 : b};
  double* gd = LDS ? Gd : Rinv;  // Rinv is written only after the factorisation
  const int tid = threadIdx.x, nt = blockDim.x;

  for (int j = tid; j < b; j += nt) gd[j] = G[j * b + j];
  __syncthreads();
  if (tid == 0) {
    double tr = 0.0;
    for (int j = 0; j < b; ++j) tr += gd[j];
    zero = !(tr > 0.0);
    shift = 0.0;
    // Fukaya shift, u = 2^-53; trace(G) >= ||U||_2^2
    if (!zero) shift = 11.0 * ((double)nglob * b + (double)b * (b + 1)) * 0x1.0p-53 * tr;
  }
  __syncthreads();

  int shifted = 0;
  if (!zero) {
    for (int attempt = 0; attempt < 2; ++attempt) {
      const double sh = attempt ? shift : 0.0;
      for (int e = tid; e < b * b; e += nt) {
        const int r = e / b, c = e % b;
        M(r, c) = (r <= c) ? G[r * b + c] + (r == c ? sh : 0.0) : 0.0;
      }
      if (tid == 0) fail = 0;
      __syncthreads();
      for (int j = 0; j < b; ++j) {
        if (tid == 0) {
          const double d = M(j, j);
          const double gjj = gd[j] + sh;
          if (!(d > 0.0) || !isfinite(d)) {
            fail = 1;
          } else {
            // relative pivot: sin^2 of the angle between u_j and span(u_<j); below 1e-15 the
            // block's condition number exceeds ~3e7 and plain CholQR2 loses orthogonality
            if (attempt == 0 && mode == 0 && d < 1e-15 * gjj) fail = 2;
            M(j, j) = sqrt(d);
          }
        }
        __syncthreads();
        if (fail) break;
        const double rjj = M(j, j);
        for (int c = j + 1 + tid; c < b; c += nt) M(j, c) /= rjj;
        __syncthreads();
        const int m = b - j - 1;
        for (int e = tid; e < m * m; e += nt) {
          const int r = j + 1 + e / m, c = j + 1 + e % m;
          if (r <= c) M(r, c) -= M(j, r) * M(j, c);
        }
        __syncthreads();
      }
      __syncthreads();
      if (!fail) break;
      shifted = 1;
      __syncthreads();
    }
  }
  __syncthreads();
  const bool bad = !zero && fail;

  // Rinv: column c by thread c (back substitution on the upper triangle)
  if (!zero && !bad) {
    for (int c = tid; c < b; c += nt) {
      for (int i = 0; i < b; ++i) X(i, c) = 0.0;
      X(c, c) = 1.0 / M(c, c);
      for (int i = c - 1; i >= 0; --i) {
        double acc = 0.0;
        for (int k = i + 1; k <= c; ++k) acc += M(i, k) * X(k, c);
        X(i, c) = -acc / M(i, i);
      }
    }
  }
  __syncthreads();
  for (int e = tid; e < b * b; e += nt) {
    const int r = e / b, c = e % b;
    const bool up = r <= c;
    const double rv = (zero || bad || !up) ? 0.0 : M(r, c);
    const double xv = (zero || bad || !up) ? 0.0 : X(r, c);
    R[e] = rv;
    Rinv[e] = xv;
  }
  __syncthreads();
  // Rtot = R * Rtot_prev (mode 1) or R (mode 0); reuse X as scratch for the product
  if (mode == 0) {
    for (int e = tid; e < b * b; e += nt) Rtot[e] = R[e];
  } else {
    for (int e = tid; e < b * b; e += nt) X(e / b, e % b) = Rtot[e];
    __syncthreads();
    for (int e = tid; e < b * b; e += nt) {
      const int r = e / b, c = e % b;
      double acc = 0.0;
      if (r <= c && !zero && !bad)
        for (int k = r; k <= c; ++k) acc += M(r, k) * X(k, c);
      Rtot[e] = acc;
    }
  }
  if (tid == 0) {
    if (mode == 0) { need3[0] = shifted; need3[1] = !shifted; }
    if (bad) status[0] = 1;
    if (shifted) status[1] += 1;
  }
}

// The same factorisation for b = 16 / 32 on ONE wave with the matrix in registers: lane c holds
// column c of M (then of R^-1, then of Rtot), and the row elements another lane holds come over
// v_readlane (lane index a compile-time constant: the loops are unrolled).  k_chol spends its
// time in ~3 four-wave barriers per column and a serial pivot on thread 0 (26 us per call at
// b = 32, ~7 calls per block step); here there is no barrier at all.  Every entry is formed
// by the same operations in the same order as k_chol (terms that k_chol skips are exact zeros
// here, added at the end of a sum), so R, R^-1 and Rtot come out the same.
__device__ __forceinline__ double bcast(double v, int lane) {
  const unsigned long long u = __builtin_bit_cast(unsigned long long, v);
  const unsigned lo = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)u, lane);
  const unsigned hi = (unsigned)__builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
  return __builtin_bit_cast(double, ((unsigned long long)hi << 32) | lo);
}

template <int B>
__global__ __launch_bounds__(64) void k_chol_reg(const double* __restrict__ G, int64_t nglob, int mode,
                                                 double* R, double* Rinv, double* Rtot, int* need3,
                                                 int* status, const int* skip) {
  if (skip && *skip) return;
  const int c = threadIdx.x;           // the column this lane holds (lanes >= B hold nothing)
  const int cc = c < B ? c : B - 1;    // clamped for loads
  double tr = 0.0;
#pragma unroll
  for (int j = 0; j < B; ++j) tr += G[j * B + j];
  const bool zero = !(tr > 0.0);
  const double shift = zero ? 0.0 : 11.0 * ((double)nglob * B + (double)B * (B + 1)) * 0x1.0p-53 * tr;
  double m[B];
  int fail = 0, shifted = 0;
  if (!zero) {
    for (int attempt = 0; attempt < 2; ++attempt) {
      const double sh = attempt ? shift : 0.0;
#pragma unroll
      for (int r = 0; r < B; ++r) m[r] = (r <= c) ? G[r * B + cc] + (r == c ? sh : 0.0) : 0.0;
      fail = 0;
#pragma unroll
      for (int j = 0; j < B; ++j) {
        const double d = bcast(m[j], j);  // M(j, j), held by lane j
        const double gjj = G[j * B + j] + sh;
        if (!(d > 0.0) || !isfinite(d)) {
          fail = 1;
        } else if (attempt == 0 && mode == 0 && d < 1e-15 * gjj) {
          fail = 2;
        }
        if (fail) break;
        const double rjj = sqrt(d);
        if (c == j) m[j] = rjj;
        if (c > j) m[j] /= rjj;            // M(j, c) /= rjj
#pragma unroll
        for (int r = j + 1; r < B; ++r) {  // M(r, c) -= M(j, r) M(j, c), r <= c
          const double mjr = bcast(m[j], r);
          if (r <= c) m[r] -= mjr * m[j];
        }
      }
      if (!fail) break;
      shifted = 1;
    }
  }
  const bool bad = !zero && fail;
  const bool ok = !zero && !bad;
  // R^-1, column c: X(c, c) = 1 / M(c, c); X(i, c) = -sum_{k = i+1..c} M(i, k) X(k, c) / M(i, i)
  double x[B];
#pragma unroll
  for (int i = 0; i < B; ++i) x[i] = 0.0;
  if (ok) {
#pragma unroll
    for (int i = B - 1; i >= 0; --i) {
      const double mii = bcast(m[i], i);
      if (i == c) x[i] = 1.0 / mii;
      double acc = 0.0;
#pragma unroll
      for (int k = i + 1; k < B; ++k) acc += bcast(m[i], k) * x[k];  // x[k] = 0 for k > c
      if (i < c) x[i] = -acc / mii;
    }
  }
  if (c < B) {
#pragma unroll
    for (int r = 0; r < B; ++r) {
      const bool up = r <= c && ok;
      R[r * B + c] = up ? m[r] : 0.0;
      Rinv[r * B + c] = up ? x[r] : 0.0;
    }
  }
  // Rtot = R (mode 0) or R Rtot_prev (mode 1), column c; Rtot_prev is upper triangular
  if (mode == 0) {
    if (c < B) {
#pragma unroll
      for (int r = 0; r < B; ++r) Rtot[r * B + c] = (r <= c && ok) ? m[r] : 0.0;
    }
  } else {
    double p[B];
#pragma unroll
    for (int k = 0; k < B; ++k) p[k] = Rtot[k * B + cc];
    __syncthreads();  // every lane has read Rtot_prev before any lane overwrites it
    double out[B];
#pragma unroll
    for (int r = 0; r < B; ++r) {
      double acc = 0.0;
#pragma unroll
      for (int k = r; k < B; ++k) acc += bcast(m[r], k) * p[k];  // p[k] = 0 for k > c
      out[r] = (r <= c && ok) ? acc : 0.0;
    }
    if (c < B) {
#pragma unroll
      for (int r = 0; r < B; ++r) Rtot[r * B + c] = out[r];
    }
  }
  if (c == 0) {
    if (mode == 0) { need3[0] = shifted; need3[1] = !shifted; }
    if (bad) status[0] = 1;
    if (shifted) status[1] += 1;
  }
}

// The same Cholesky on one wave with R^-1 formed in the same sweep: every row operation of the
// right-looking factorisation (row j scaled by 1 / r_jj, row r minus M(j, r) times row j) is also
// applied to X = I, which therefore ends as R^-T — no separate back substitution, whose 32
// dependent divisions and sums made up half of k_chol_reg's time.  Row j goes to the other lanes
// through LDS (a wave's LDS operations complete in issue order: one write, then broadcast reads;
// no barrier), and R is staged in LDS once for the Rtot product.  R and Rtot have k_chol's bits;
// R^-1 differs from the back substitution's at rounding level (both paths of every comparison in
// the tests run this kernel).
template <int B>
__global__ __launch_bounds__(64) void k_chol_elim(const double* __restrict__ G, int64_t nglob, int mode,
                                                  double* R, double* Rinv, double* Rtot, int* need3,
                                                  int* status, const int* skip) {
  if (skip && *skip) return;
  __shared__ double rowj[2][64];
  __shared__ __attribute__((aligned(16))) double Ms[B][B + 2];
  const int c = threadIdx.x;
  const int cc = c < B ? c : B - 1;
  double tr = 0.0;
#pragma unroll
  for (int j = 0; j < B; ++j) tr += G[j * B + j];
  const bool zero = !(tr > 0.0);
  const double shift = zero ? 0.0 : 11.0 * ((double)nglob * B + (double)B * (B + 1)) * 0x1.0p-53 * tr;
  double m[B], x[B];
  int fail = 0, shifted = 0;
  if (!zero) {
    for (int attempt = 0; attempt < 2; ++attempt) {
      const double sh = attempt ? shift : 0.0;
#pragma unroll
      for (int r = 0; r < B; ++r) {
        m[r] = (r <= c) ? G[r * B + cc] + (r == c ? sh : 0.0) : 0.0;
        x[r] = r == c ? 1.0 : 0.0;
      }
      fail = 0;
#pragma unroll
      for (int j = 0; j < B; ++j) {
        const double d = bcast(m[j], j);  // M(j, j), held by lane j
        const double gjj = G[j * B + j] + sh;
        if (!(d > 0.0) || !isfinite(d)) {
          fail = 1;
        } else if (attempt == 0 && mode == 0 && d < 1e-15 * gjj) {
          fail = 2;
        }
        if (fail) break;
        const double rjj = sqrt(d);
        if (c == j) m[j] = rjj;
        if (c > j) m[j] /= rjj;  // M(j, c) /= rjj
        x[j] /= rjj;             // row j of X (zero for c > j)
        if (j + 1 < B) {
          rowj[j & 1][c] = m[j];  // row j of M to every lane
          __builtin_amdgcn_wave_barrier();
#pragma unroll
          for (int r = j + 1; r < B; ++r) {
            const double mjr = rowj[j & 1][r];
            if (r <= c) m[r] -= mjr * m[j];  // M(r, c) -= M(j, r) M(j, c)
            x[r] -= mjr * x[j];              // X(r, c) -= M(j, r) X(j, c)
          }
        }
      }
      if (!fail) break;
      shifted = 1;
    }
  }
  const bool bad = !zero && fail;
  const bool ok = !zero && !bad;
  if (c < B) {
#pragma unroll
    for (int r = 0; r < B; ++r) {
      const bool up = r <= c && ok;
      R[r * B + c] = up ? m[r] : 0.0;
      Rinv[c * B + r] = (ok && r >= c) ? x[r] : 0.0;  // R^-1 (c, r) = X(r, c)
    }
  }
  if (mode == 0) {
    if (c < B) {
#pragma unroll
      for (int r = 0; r < B; ++r) Rtot[r * B + c] = (r <= c && ok) ? m[r] : 0.0;
    }
  } else {
    // Rtot = R Rtot_prev, column c: sum_{k = r..c} R(r, k) Rtot_prev(k, c) (Rtot_prev upper
    // triangular: the terms past c are exact zeros), R(r, k) broadcast from LDS
    double p[B];
#pragma unroll
    for (int k = 0; k < B; ++k) p[k] = Rtot[k * B + cc];
    if (c < B) {
#pragma unroll
      for (int r = 0; r < B; ++r) Ms[r][c] = m[r];
    }
    __syncthreads();  // one wave: R staged, and every lane has read Rtot_prev
    double out[B];
#pragma unroll
    for (int r = 0; r < B; ++r) {
      double acc = 0.0;
#pragma unroll
      for (int k = r; k < B; ++k) acc += Ms[r][k] * p[k];
      out[r] = (r <= c && ok) ? acc : 0.0;
    }
    if (c < B) {
#pragma unroll
      for (int r = 0; r < B; ++r) Rtot[r * B + c] = out[r];
    }
  }
  if (c == 0) {
    if (mode == 0) { need3[0] = shifted; need3[1] = !shifted; }
    if (bad) status[0] = 1;
    if (shifted) status[1] += 1;
  }
}

// k_chol_elim with the wave's other half at work: lanes [0, B) hold the columns of M, lanes
// [B, 2B) those of X (= I, ending as R^-T), so a column step is one division and 31 - j fused
// updates per lane instead of two and 2 (31 - j).  Every value is formed by the same operations
// in the same order as k_chol_elim: the same bits.
template <int B>
__global__ __launch_bounds__(64) void k_chol_elim2(const double* __restrict__ G, int64_t nglob, int mode,
                                                   double* R, double* Rinv, double* Rtot, int* need3,
                                                   int* status, const int* skip) {
  static_assert(2 * B <= 64, "two columns per lane pair");
  if (skip && *skip) return;
  __shared__ double rowj[2][B];
  __shared__ __attribute__((aligned(16))) double Ms[B][B + 2];
  const int c = threadIdx.x;
  const bool isx = c >= B;                            // an X lane (or idle, c >= 2B)
  const bool live = c < 2 * B;
  const int col = c < B ? c : (live ? c - B : B - 1);  // the column this lane holds
  double tr = 0.0;
#pragma unroll
  for (int j = 0; j < B; ++j) tr += G[j * B + j];
  const bool zero = !(tr > 0.0);
  const double shift = zero ? 0.0 : 11.0 * ((double)nglob * B + (double)B * (B + 1)) * 0x1.0p-53 * tr;
  double v[B];
  int fail = 0, shifted = 0;
  if (!zero) {
    for (int attempt = 0; attempt < 2; ++attempt) {
      const double sh = attempt ? shift : 0.0;
#pragma unroll
      for (int r = 0; r < B; ++r) {  // loads on every lane, then selects: no branches
        const double g = G[r * B + col];
        v[r] = isx ? (r == col ? 1.0 : 0.0) : g + (r == col ? sh : 0.0);
      }
      fail = 0;
#pragma unroll
      for (int j = 0; j < B; ++j) {
        const double d = bcast(v[j], j);  // M(j, j), held by lane j
        const double gjj = G[j * B + j] + sh;
        if (!(d > 0.0) || !isfinite(d)) {
          fail = 1;
        } else if (attempt == 0 && mode == 0 && d < 1e-15 * gjj) {
          fail = 2;
        }
        if (fail) break;
        const double rjj = sqrt(d);
        // M lanes: M(j, c) /= rjj right of the diagonal, r_jj on it; X lanes: X(j, c) /= rjj
        const double q = v[j] / rjj;
        v[j] = (!isx && col == j) ? rjj : q;
        if (j + 1 < B) {
          if (!isx) rowj[j & 1][col] = v[j];  // row j of M to every lane
          __builtin_amdgcn_wave_barrier();
          // M(r, c) or X(r, c) -= M(j, r) (.)(j, c), every r on every lane: an M lane's entries
          // below its diagonal (r > c) take values nothing reads (R, the rows sent through rowj
          // and the Rtot product use only r <= c), so no lane masks are kept across the sweep
#pragma unroll
          for (int r = j + 1; r < B; ++r) {
            const double mjr = rowj[j & 1][r];
            v[r] -= mjr * v[j];
          }
        }
      }
      if (!fail) break;
      shifted = 1;
    }
  }
  const bool bad = !zero && fail;
  const bool ok = !zero && !bad;
  if (live) {
#pragma unroll
    for (int r = 0; r < B; ++r) {
      if (!isx) R[r * B + col] = (r <= col && ok) ? v[r] : 0.0;
      else Rinv[col * B + r] = (ok && r >= col) ? v[r] : 0.0;  // R^-1 (c, r) = X(r, c)
    }
  }
  if (mode == 0) {
    if (!isx) {
#pragma unroll
      for (int r = 0; r < B; ++r) Rtot[r * B + col] = (r <= col && ok) ? v[r] : 0.0;
    }
  } else {
    // Rtot = R Rtot_prev, column c: sum_{k = r..c} R(r, k) Rtot_prev(k, c) on the M lanes (the
    // terms past c are exact zeros), R(r, k) broadcast from LDS
    double p[B];
#pragma unroll
    for (int k = 0; k < B; ++k) p[k] = Rtot[k * B + col];
    if (!isx) {
#pragma unroll
      for (int r = 0; r < B; ++r) Ms[r][col] = v[r];
    }
    __syncthreads();  // one wave: R staged, and every lane has read Rtot_prev
    if (!isx) {
#pragma unroll
      for (int r = 0; r < B; ++r) {
        double acc = 0.0;
#pragma unroll
        for (int k = r; k < B; ++k) acc += Ms[r][k] * p[k];
        Rtot[r * B + col] = (r <= col && ok) ? acc : 0.0;
      }
    }
  }
  if (c == 0) {
    if (mode == 0) { need3[0] = shifted; need3[1] = !shifted; }
    if (bad) status[0] = 1;
    if (shifted) status[1] += 1;
  }
}

// RBL_CHOL_REG: 0 the four-wave kernel at b = 16 / 32 as well, 1 k_chol_reg, 2 k_chol_elim2
// (default), 3 k_chol_elim (the one-half-wave form, same bits as 2)
// (A/B; read per call, tests switch it)
#ifdef RBL_VARIANTS
static int chol_reg_mode() {
  const char* e = getenv("RBL_CHOL_REG");
  return e ? atoi(e) : 2;
}
#else
// the product build: k_chol_elim2 at b = 16 / 32, the four-wave kernel for any other b
static constexpr int chol_reg_mode() { return 2; }
#endif

void chol_step(const double* G, int b, int64_t nglobal, int mode, double* R, double* Rinv,
               double* Rtot, int* need3, int* status, const int* skip, hipStream_t s,
               double* scratch) {
  const int cm = (b == 32 || b == 16) ? chol_reg_mode() : 0;
  if (cm == 2) {
    if (b == 32)
      hipLaunchKernelGGL(k_chol_elim2<32>, dim3(1), dim3(64), 0, s, G, nglobal, mode, R, Rinv, Rtot,
                         need3, status, skip);
    else
      hipLaunchKernelGGL(k_chol_elim2<16>, dim3(1), dim3(64), 0, s, G, nglobal, mode, R, Rinv, Rtot,
                         need3, status, skip);
    return;
  }
#ifdef RBL_VARIANTS
  if (cm == 3) {
    if (b == 32)
      hipLaunchKernelGGL(k_chol_elim<32>, dim3(1), dim3(64), 0, s, G, nglobal, mode, R, Rinv, Rtot,
                         need3, status, skip);
    else
      hipLaunchKernelGGL(k_chol_elim<16>, dim3(1), dim3(64), 0, s, G, nglobal, mode, R, Rinv, Rtot,
                         need3, status, skip);
    return;
  }
  if (cm == 1) {
    if (b == 32)
      hipLaunchKernelGGL(k_chol_reg<32>, dim3(1), dim3(64), 0, s, G, nglobal, mode, R, Rinv, Rtot,
                         need3, status, skip);
    else
      hipLaunchKernelGGL(k_chol_reg<16>, dim3(1), dim3(64), 0, s, G, nglobal, mode, R, Rinv, Rtot,
                         need3, status, skip);
    return;
  }
#endif
  if (b <= kMaxB)
    hipLaunchKernelGGL(k_chol<true>, dim3(1), dim3(256), 0, s, G, b, nglobal, mode, R, Rinv, Rtot,
                       need3, status, skip, scratch);
  else
    hipLaunchKernelGGL(k_chol<false>, dim3(1), dim3(256), 0, s, G, b, nglobal, mode, R, Rinv, Rtot,
                       need3, status, skip, scratch);
}

__global__ void k_copy(const double* __restrict__ src, double* __restrict__ dst, int64_t len,
                       const int* skip) {
  if (skip && *skip) return;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < len;
       e += (int64_t)gridDim.x * blockDim.x)
    dst[e] = src[e];
}
void copy_small(const double* src, double* dst, int64_t len, hipStream_t s, const int* skip) {
  int64_t blocks = (len + 255) / 256;
  if (blocks > 8192) blocks = 8192;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(k_copy, dim3((unsigned)blocks), dim3(256), 0, s, src, dst, len, skip);
}

// End of a block step: A_i, R_tot (= B_{i+1}) and the four step flags into one contiguous
// record for a single D2H copy, R_tot into B_prev for the next step's 3-term epilogue, and the
// flags cleared for the next step — one launch where a copy kernel, three small D2H copies (a
// blit each) and the next step's flag memset ran.
__global__ void k_stash(const double* __restrict__ Ai, const double* __restrict__ Rtot,
                        double* __restrict__ Bprev, int* __restrict__ flags,
                        double* __restrict__ stash, int bb) {
  for (int e = threadIdx.x; e < bb; e += blockDim.x) {
    stash[e] = Ai[e];
    const double r = Rtot[e];
    stash[bb + e] = r;
    Bprev[e] = r;
  }
  if (threadIdx.x < 4) {
    reinterpret_cast<int*>(stash + 2 * bb)[threadIdx.x] = flags[threadIdx.x];
    flags[threadIdx.x] = 0;
  }
  __threadfence_system();  // the record may be coherent host memory, read after the step's event
}
void stash_step(const double* Ai, const double* Rtot, double* Bprev, int* flags, double* stash,
                int b, hipStream_t s) {
  hipLaunchKernelGGL(k_stash, dim3(1), dim3(256), 0, s, Ai, Rtot, Bprev, flags, stash, b * b);
}

// C = C R^-1 (b x b row-major, R^-1 upper triangular) unless *skip: the next step's local-reorth
// Gram Z^T Q after CholQR's third pass (Q3 = Q2 R3^-1, so Z^T Q3 = (Z^T Q2) R3^-1), formed from
// the pass-2 Gram already all-reduced instead of a fourth collective
__global__ void k_cloc_rinv(double* __restrict__ C, const double* __restrict__ Rinv, int b,
                            const int* __restrict__ skip) {
  if (skip && *skip) return;
  __shared__ double c[kMaxB * kMaxB];
  const int bb = b * b;
  for (int e = threadIdx.x; e < bb; e += blockDim.x) c[e] = C[e];
  __syncthreads();
  for (int e = threadIdx.x; e < bb; e += blockDim.x) {
    const int r = e / b, col = e % b;
    double acc = 0.0;
    for (int k = 0; k <= col; ++k) acc += c[r * b + k] * Rinv[k * b + col];
    C[e] = acc;
  }
}
void cloc_rinv(double* C, const double* Rinv, int b, const int* skip, hipStream_t s) {
  if (getenv("RBL_DIAG_CLOC_NOFIX")) return;  // diagnostics: the test's negative control
  hipLaunchKernelGGL(k_cloc_rinv, dim3(1), dim3(256), 0, s, C, Rinv, b, skip);
}

// dst = src^T (b x b row-major): B_i^T for the dense path's 3-term epilogue
__global__ void k_transpose_small(const double* __restrict__ src, double* __restrict__ dst, int b) {
  for (int e = threadIdx.x; e < b * b; e += blockDim.x) dst[(e % b) * b + e / b] = src[e];
}
void transpose_small(const double* src, double* dst, int b, hipStream_t s) {
  hipLaunchKernelGGL(k_transpose_small, dim3(1), dim3(256), 0, s, src, dst, b);
}

}  // namespace rbl
