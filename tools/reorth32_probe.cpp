// reorth32_probe.cpp — time the shipped fp32-basis partial-reorth kernels (gram32_partial +
// reduce_slab, tsmm32) at n = 1e7, b = 32, X = [Q_i, Q_{i-1}] for a range of basis sizes
// (diagnostic, the fp32 twin of reorth_probe.cpp).  Build: tools/build_probe.sh.
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#include "../gpu-randomized-block-lanczos_amd/csrc/kernels.hpp"

__global__ void k_fillf(float* p, int64_t n, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    p[i] = (float)(((double)(z >> 11) * 0x1.0p-53 - 0.5) * 1e-2);
  }
}
__global__ void k_filld(double* p, int64_t n, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    p[i] = (double)((i * 2654435761ull + seed) % 1000) * 1e-5;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 10000000;
  const int b = 32, nWmax = 36;
  float *W, *X0, *X1;
  double *slab, *C, *Cg;
  if (hipMalloc(&W, (size_t)n * b * nWmax * 4) != hipSuccess) return 1;
  (void)hipMalloc(&X0, (size_t)n * b * 4);
  (void)hipMalloc(&X1, (size_t)n * b * 4);
  hipLaunchKernelGGL(k_fillf, dim3(4096), dim3(256), 0, 0, W, n * b * nWmax, 1);
  hipLaunchKernelGGL(k_fillf, dim3(4096), dim3(256), 0, 0, X0, n * b, 2);
  hipLaunchKernelGGL(k_fillf, dim3(4096), dim3(256), 0, 0, X1, n * b, 3);
  const int splits = rbl::gram32_splits(n);
  (void)hipMalloc(&slab, (size_t)splits * nWmax * b * 64 * 8);
  (void)hipMalloc(&C, (size_t)nWmax * b * 64 * 8);
  hipLaunchKernelGGL(k_filld, dim3(256), dim3(256), 0, 0, C, (int64_t)nWmax * b * 64, 4);
  (void)hipMalloc(&Cg, (size_t)nWmax * b * 64 * 8);
  hipEvent_t e0, e1, e2;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventCreate(&e2);
  double tg = 0, tt = 0, fl = 0;
  for (int nW = 2; nW <= nWmax; nW += 2) {
    float bg = 1e30f, bt = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      // PROBE_W0=1: every panel aliases panel 0 (basis from cache, same instructions)
      const int64_t ws = (getenv("PROBE_W0") && atoi(getenv("PROBE_W0"))) ? 0 : n * b;
      rbl::gram32_partial(n, W, ws, nW, b, X0, X1, 2, slab, splits, 0);
      rbl::reduce_slab(slab, splits, (int64_t)nW * b * 64, Cg, nullptr, 0);
      (void)hipEventRecord(e1);
      rbl::tsmm32(n, W, ws, nW, b, C, 64, X0, X1, 2, -1.f, 1.f, 0);
      (void)hipEventRecord(e2);
      (void)hipEventSynchronize(e2);
      float g, t;
      (void)hipEventElapsedTime(&g, e0, e1);
      (void)hipEventElapsedTime(&t, e1, e2);
      if (rep) {
        bg = g < bg ? g : bg;
        bt = t < bt ? t : bt;
      }
    }
    const double f = 2.0 * n * nW * b * 64;
    printf("nW=%2d  gram32 %7.3f ms %6.1f TF   tsmm32 %7.3f ms %6.1f TF\n", nW, bg, f / bg / 1e9, bt,
           f / bt / 1e9);
    tg += bg;
    tt += bt;
    fl += f;
  }
  printf("sum over nW=2..36 step 2: gram32 %.1f ms (%.1f TF)  tsmm32 %.1f ms (%.1f TF)\n", tg,
         fl / tg / 1e9, tt, fl / tt / 1e9);
  return 0;
}
