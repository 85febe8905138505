// tsmm_probe.hip — k_tsmm44<32,64> (reorth.hip) variants: MODE bit 0 drops the per-chunk
// barrier (wrong results; upper bound), WPE = amdgpu_waves_per_eu (diagnostic).
#include "../gpu-randomized-block-lanczos_amd/csrc/kernels.hpp"
#include <cstdio>
using namespace rbl;
__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
__global__ void k_fill(double* p, int64_t n, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    p[i] = ((double)(z >> 11) * 0x1.0p-53 - 0.5) * 1e-2;
  }
}
constexpr int kT44Rows = 32;   // rows per wave
constexpr int kT44K = 32;      // k per chunk

template <int B, int KYP, int MODE, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE))) void k_tsmm44(int64_t nrows, PanelRun X, const double* __restrict__ C,
                                                int ldc, int KY, Panels Y, double alpha, double beta,
                                                const int* skip) {
  if (skip && *skip) return;
  constexpr int CG = KYP / 4;
  constexpr int LDC = KYP + 8;  // lane-group rows differ by 2: LDC = 8 mod 16 (see k_gram44)
  __shared__ __attribute__((aligned(16))) double cs[2][kT44K * LDC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * kT44Rows;
  const int K = X.count * B;
  const int nch = (K + kT44K - 1) / kT44K;

  double acc[2][CG];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int cg = 0; cg < CG; ++cg) acc[rt][cg] = 0.0;

  // Y rows for beta != 0, row-major 16 B per lane (element e = 2 lane + 128 m of each
  // 16-row tile), loaded before the k-loop so their latency hides behind it
  constexpr int kYPer = 16 * KYP / 128;
  constexpr bool kPrefY = KYP <= 32;  // b x b updates (one k-chunk); long-K runs load Y late
  d2v yold[2][kYPer];
  auto load_y = [&](int rt, int m) -> d2v {
    const int e = 2 * lane + 128 * m, row = e / KYP, c = e % KYP;
    int64_t r = r0 + 16 * rt + row;
    r = r < nrows ? r : nrows - 1;
    const int cc = c < KY ? c : 0;
    const int t = cc / Y.w;
    return *reinterpret_cast<const d2v*>(Y.ptr[t] + r * Y.w + (cc - t * Y.w));
  };
  if (kPrefY && beta != 0.0) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int m = 0; m < kYPer; ++m) yold[rt][m] = load_y(rt, m);
  }

  // A: rows r0 + 16 rt + (lane&15); k = k0 + 8 h + 2 q + v, h in [0,4), v in {0,1}
  // Prefetch loads are unconditional (clamped addresses) so each chunk issues the same VMEM
  // ops and the vmcnt waits count only the chunk consumed.  Rows past nrows compute garbage
  // that is never stored; k past K reads a valid panel but meets zeroed C rows (zeroed at
  // the LDS store).
  int64_t arow[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int64_t r = r0 + 16 * rt + (lane & 15);
    arow[rt] = r < nrows ? r : nrows - 1;
  }
  auto load_a = [&](int ch, d2v (&ar)[2][4]) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int k0 = ch * kT44K + 8 * h + 2 * q;
      const int k = k0 < K ? k0 : K - 2;
      const int pan = k / B;
      const int col = k - pan * B;
      const double* xp = X.base + (int64_t)pan * X.stride + col;
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) ar[rt][h] = *reinterpret_cast<const d2v*>(xp + arow[rt] * B);
    }
  };
  // C chunk: 32 x KYP, 256 threads; element e -> (k = e / KYP, c = e % KYP)
  constexpr int CEPT = kT44K * KYP / 256;
  auto load_c = [&](int ch, double (&cr)[CEPT]) {
#pragma unroll
    for (int v = 0; v < CEPT; ++v) {
      const int e = tid + v * 256;
      const int k = ch * kT44K + e / KYP, c = e % KYP;
      const int kc = k < K ? k : K - 1, cc = c < KY ? c : KY - 1;
      cr[v] = C[(int64_t)kc * ldc + cc];
    }
  };
  auto store_c = [&](int buf, int ch, const double (&cr)[CEPT]) {
#pragma unroll
    for (int v = 0; v < CEPT; ++v) {
      const int e = tid + v * 256;
      const int k = ch * kT44K + e / KYP, c = e % KYP;
      cs[buf][(e / KYP) * LDC + perm8(e % KYP)] = (k < K && c < KY) ? cr[v] : 0.0;
    }
  };

  d2v acur[2][4], anext[2][4];
  double cr[CEPT];
  load_c(0, cr);
  store_c(0, 0, cr);
  load_a(0, acur);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    load_c(ch + 1, cr);  // unconditional, clamped (see k_gram44)
    load_a(ch + 1, anext);
    const double* cb = cs[ch & 1] + 2 * q * LDC + 2 * (lane & 3);
#pragma unroll
    for (int hv = 0; hv < 8; ++hv) {
      const int h = hv >> 1, v = hv & 1;
      const double* cr0 = cb + (8 * h + v) * LDC;
#pragma unroll
      for (int cp = 0; cp < CG / 2; ++cp) {  // column groups 2cp, 2cp+1 in one 16-B read
        const d2v bf = *reinterpret_cast<const d2v*>(cr0 + 8 * cp);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
          acc[rt][2 * cp] = mfma4(acur[rt][h][v], bf.x, acc[rt][2 * cp]);
          acc[rt][2 * cp + 1] = mfma4(acur[rt][h][v], bf.y, acc[rt][2 * cp + 1]);
        }
      }
    }
    store_c((ch + 1) & 1, ch + 1, cr);  // unconditional (see k_gram44)
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int h = 0; h < 4; ++h) acur[rt][h] = anext[rt][h];
    if (!(MODE & 1)) __syncthreads();
  }
  // epilogue: the D-layout tile goes through LDS (the C buffers are free after the loop's
  // last barrier) so Y is read and written row-major, 16 B per lane, fully coalesced; Y was
  // prefetched before the k-loop.  Column c of staged row r sits at c ^ (4 ((r >> 2) & 3)):
  // the four row quads a ds_write_b64 lane group covers land 8 banks apart.
  double* ot = &cs[0][0] + wave * 16 * KYP;
  const int g = (lane >> 2) & 3;
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
#pragma unroll
    for (int cg = 0; cg < CG; ++cg)
      ot[(4 * g + q) * KYP + ((4 * cg + (lane & 3)) ^ (4 * g))] = alpha * acc[rt][cg];
#pragma unroll
    for (int m = 0; m < kYPer; ++m) {
      const int e = 2 * lane + 128 * m, row = e / KYP, c = e % KYP;
      const int64_t r = r0 + 16 * rt + row;
      d2v v = *reinterpret_cast<const d2v*>(ot + row * KYP + (c ^ (4 * ((row >> 2) & 3))));
      if (r < nrows && c < KY) {
        const int t = c / Y.w;
        d2v* yp = reinterpret_cast<d2v*>(const_cast<double*>(Y.ptr[t]) + r * Y.w + (c - t * Y.w));
        if (beta != 0.0) v += beta * (kPrefY ? yold[rt][m] : load_y(rt, m));
        *yp = v;
      }
    }
  }
}


template <int MODE, int WPE>
void run(const char* name, int64_t n, const PanelRun& X, const double* C, const Panels& Y) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  float best = 1e30f;
  const int64_t wgs = (n + 4 * kT44Rows - 1) / (4 * kT44Rows);
  for (int rep = 0; rep < 3; ++rep) {
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL((k_tsmm44<32, 64, MODE, WPE>), dim3((unsigned)wgs), dim3(256), 0, 0, n, X, C, 64,
                       64, Y, -1.0, 1.0, nullptr);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    if (rep && ms < best) best = ms;
  }
  printf("%-14s WPE=%d nW=%2d: %7.3f ms %5.1f TF\n", name, WPE, X.count, best,
         2.0 * n * X.count * 32 * 64 / best / 1e9);
}
int main() {
  const int64_t n = 10000000;
  const int nWmax = 36;
  double *W, *Y0, *Y1, *C;
  if (hipMalloc(&W, (size_t)n * 32 * nWmax * 8) != hipSuccess) return 1;
  (void)hipMalloc(&Y0, (size_t)n * 32 * 8);
  (void)hipMalloc(&Y1, (size_t)n * 32 * 8);
  (void)hipMalloc(&C, (size_t)nWmax * 32 * 64 * 8);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, W, n * 32 * nWmax, 1);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, Y0, n * 32, 2);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, Y1, n * 32, 3);
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, C, nWmax * 32 * 64, 4);
  Panels Y;
  Y.ptr[0] = Y0;
  Y.ptr[1] = Y1;
  Y.count = 2;
  Y.w = 32;
  for (int nW : {4, 18, 36}) {
    PanelRun X;
    X.base = W;
    X.stride = n * 32;
    X.count = nW;
    X.w = 32;
    run<0, 3>("shipped", n, X, C, Y);
    run<1, 3>("no barrier", n, X, C, Y);
    run<0, 2>("shipped", n, X, C, Y);
    run<1, 2>("no barrier", n, X, C, Y);
  }
  return 0;
}
