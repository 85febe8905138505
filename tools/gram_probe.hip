// gram_probe.hip — what keeps k_gram44<32,2> (partial-reorth Gram W^T X, reorth.hip) below the
// 4x4x4 fp64 MFMA ceiling?  The same loop structure with components switched off (diagnostic):
//   MODE bit 0: no W global loads (A operands from registers)
//   MODE bit 1: no LDS B reads (B operands from registers)
//   MODE bit 2: no X staging (no X global loads / LDS stores)
//   MODE bit 3: no per-chunk barrier
// AG = 16-column W groups per wave (2: one 32-wide panel per wave, as shipped; 4: two panels).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

typedef double d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ int perm8(int c) { return (c & ~7) | ((c & 3) << 1) | ((c >> 2) & 1); }
__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

constexpr int kRows = 32;
constexpr int B = 32;

template <int MODE, int AG, int ROWS, int WAVES>
__global__ __launch_bounds__(WAVES * 64) void k_g(int64_t nrows, const double* W, int64_t wstride, int nW,
                                           const double* X0, const double* X1, double* slab,
                                           int npg, int64_t rows_per) {
  constexpr int KC = 64;
  constexpr int CG = KC / 4;
  constexpr int LD = KC + 8;
  constexpr int EPT = ROWS * KC / (WAVES * 64);
  constexpr int KS = ROWS / 4;
  constexpr int PPW = AG / 2;  // panels per wave
  __shared__ __attribute__((aligned(16))) double xs[2][ROWS * LD];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4;
  const int bid = blockIdx.x;
  const int xcd = bid & 7, t = bid >> 3;
  const int pg = t % npg;
  const int64_t s = (int64_t)(t / npg) * 8 + xcd;
  const int64_t r_begin = s * rows_per;
  const int64_t r_end = r_begin + rows_per < nrows ? r_begin + rows_per : nrows;
  const int j = (pg * WAVES + wave) * PPW;
  const bool active = j < nW;
  const double* wp = W + (int64_t)(active ? j : 0) * wstride + (lane & 15);

  double acc[AG][CG];
#pragma unroll
  for (int ag = 0; ag < AG; ++ag)
#pragma unroll
    for (int cg = 0; cg < CG; ++cg) acc[ag][cg] = 0.0;

  const int xe0 = tid * EPT;
  const int xrow = xe0 / KC, xcol = xe0 % KC;
  const double* xsrc = (xcol < B ? X0 : X1) + (xcol % B);
  const int64_t rlast = r_end > 0 ? r_end - 1 : 0;
  auto load_x = [&](int64_t rc0, double (&xr)[EPT]) {
    const int64_t r = rc0 + xrow;
    const int64_t rc = r < rlast ? r : rlast;
#pragma unroll
    for (int v = 0; v < EPT; ++v) xr[v] = xsrc[rc * B + v];
  };
  auto store_x = [&](int buf, int64_t rc0, const double (&xr)[EPT]) {
    const bool ok = rc0 + xrow < r_end;
#pragma unroll
    for (int v = 0; v < EPT; ++v) xs[buf][xrow * LD + perm8(xcol + v)] = ok ? xr[v] : 0.0;
  };
  auto load_a = [&](int64_t rc0, double (&ar)[KS][AG]) {
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int64_t r = rc0 + 4 * ks + q;
      const int64_t rc = r < rlast ? r : rlast;
#pragma unroll
      for (int ag = 0; ag < AG; ++ag)
        ar[ks][ag] = wp[(ag / 2) * wstride + ((MODE & 1) ? (rc & 31) : rc) * B + 16 * (ag & 1)];
    }
  };

  const int64_t nchunks = r_end > r_begin ? (r_end - r_begin + ROWS - 1) / ROWS : 0;
  double xr[EPT];
  double acur[KS][AG], anext[KS][AG];
  if (nchunks > 0) {
    if (!(MODE & 4)) {
      load_x(r_begin, xr);
      store_x(0, r_begin, xr);
    }
    load_a(r_begin, acur);
  }
  __syncthreads();
  for (int64_t c = 0; c < nchunks; ++c) {
    const int64_t rc0 = r_begin + c * ROWS;
    if (!(MODE & 4)) load_x(rc0 + ROWS, xr);
    load_a(rc0 + ROWS, anext);
    const double* xb = xs[c & 1];
    if (active) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
        for (int cp = 0; cp < CG / 2; ++cp) {
          d2v bf;
          if (MODE & 2) {
            bf.x = 1.0 + ks * 1e-3 + cp;
            bf.y = 2.0 - ks * 1e-3 + cp;
          } else {
            bf = *reinterpret_cast<const d2v*>(xb + (4 * ks + q) * LD + 8 * cp + 2 * (lane & 3));
          }
#pragma unroll
          for (int ag = 0; ag < AG; ++ag) {
            acc[ag][2 * cp] = mfma4(acur[ks][ag], bf.x, acc[ag][2 * cp]);
            acc[ag][2 * cp + 1] = mfma4(acur[ks][ag], bf.y, acc[ag][2 * cp + 1]);
          }
        }
      }
    }
    if (!(MODE & 4)) store_x((int)((c + 1) & 1), rc0 + ROWS, xr);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int ag = 0; ag < AG; ++ag) acur[ks][ag] = anext[ks][ag];
    if (!(MODE & 8)) __syncthreads();
  }
  if (!active) return;
  double* out = slab + ((s * nW + j) * B) * KC;
  const int g = (lane >> 2) & 3;
#pragma unroll
  for (int ag = 0; ag < AG; ++ag)
#pragma unroll
    for (int cg = 0; cg < CG; ++cg) {
      const int a = 16 * ag + 4 * g + (lane >> 4);
      const int cc = 4 * cg + (lane & 3);
      out[(int64_t)a * KC + cc] = acc[ag][cg];
    }
}

template <int MODE, int AG, int ROWS, int WAVES = 8>
void run(const char* name, int64_t n, const double* W, int nW, const double* X0, const double* X1,
         double* slab, int splits) {
  const int ppw = AG / 2;
  const int npg = (nW + WAVES * ppw - 1) / (WAVES * ppw);
  int64_t rows_per = (n + splits - 1) / splits;
  rows_per = (rows_per + ROWS - 1) / ROWS * ROWS;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_g<MODE, AG, ROWS, WAVES>), dim3(npg * splits), dim3(WAVES * 64), 0, 0, n, W, n * B, nW,
                       X0, X1, slab, npg, rows_per);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep && ms < best) best = ms;
  }
  const double flops = 2.0 * n * (double)nW * B * 64;
  const double bytes = 8.0 * n * ((double)nW * B + 64);
  printf("%-22s nW=%2d waves=%d AG=%d rows=%d: %8.3f ms  %6.1f TF/s  %6.2f TB/s\n", name, nW, WAVES, AG, ROWS, best,
         flops / best / 1e9, bytes / best / 1e9);
}

int main() {
  const int64_t n = 10000000;
  const int nWmax = 32;
  double *W, *X0, *X1, *slab;
  if (hipMalloc(&W, (size_t)n * B * nWmax * 8) != hipSuccess) return 1;
  (void)hipMalloc(&X0, (size_t)n * B * 8);
  (void)hipMalloc(&X1, (size_t)n * B * 8);
  (void)hipMemset(W, 0, (size_t)n * B * nWmax * 8);
  (void)hipMemset(X0, 0, (size_t)n * B * 8);
  (void)hipMemset(X1, 0, (size_t)n * B * 8);
  (void)hipMalloc(&slab, (size_t)1024 * nWmax * B * 64 * 8);
  for (int nW : {16, 18, 32}) {
    run<0, 2, 32, 8>("shipped", n, W, nW, X0, X1, slab, 256);
    run<8, 2, 32, 8>("no barrier", n, W, nW, X0, X1, slab, 256);
    run<1, 2, 32, 8>("W from L2", n, W, nW, X0, X1, slab, 256);
    run<0, 2, 32, 4>("4 waves, 512 splits", n, W, nW, X0, X1, slab, 512);
    run<0, 2, 32, 4>("4 waves, 768 splits", n, W, nW, X0, X1, slab, 768);
    run<8, 2, 32, 4>("4w no barrier", n, W, nW, X0, X1, slab, 768);
    run<1, 2, 32, 4>("4w W from L2", n, W, nW, X0, X1, slab, 768);
    run<0, 2, 16, 4>("4 waves, 768 splits", n, W, nW, X0, X1, slab, 768);
  }
  return 0;
}
