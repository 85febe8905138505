// mfma_power_probe.hip — sustained v_mfma_f64_4x4x4f64 rate when the operands change every
// instruction (random mantissas, as in the partial-reorth GEMMs) vs fixed operands (as in
// tools/mfma_probe.hip).  Separates the issue-rate ceiling from a power/clock ceiling
// (diagnostic).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

__device__ __forceinline__ double rnd(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  z ^= z >> 31;
  return ((double)(z >> 11) * 0x1.0p-53 - 0.5) * 1e-2;
}

// RANDOM = 0: a, b fixed per lane; 1: 16 random a and 16 random b per lane, rotated each step
template <int RANDOM>
__global__ __launch_bounds__(256) void k_mfma(double* out, int iters) {
  double av[16], bv[16];
  const uint64_t t = blockIdx.x * 256ull + threadIdx.x;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    av[i] = RANDOM ? rnd(t * 64 + i) : 0.5 + t * 1e-9;
    bv[i] = RANDOM ? rnd(t * 64 + 32 + i) : 1.0 - t * 1e-9;
  }
  double acc[16];
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int k = 0; k < 16; ++k)
#pragma unroll
      for (int i = 0; i < 16; ++i)
        acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(av[(i + k) & 15], bv[(3 * i + k) & 15], acc[i], 0, 0, 0);
  }
  double s = 0;
#pragma unroll
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[t] = s;
}

int main() {
  double* out;
  (void)hipMalloc(&out, 1 << 26);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 2000;
  for (int wgs : {256 * 4, 256 * 8}) {
    for (int r = 0; r < 2; ++r) {
      float best = 1e30f;
      for (int rep = 0; rep < 3; ++rep) {
        (void)hipEventRecord(e0);
        if (r) hipLaunchKernelGGL(k_mfma<1>, dim3(wgs), dim3(256), 0, 0, out, iters);
        else hipLaunchKernelGGL(k_mfma<0>, dim3(wgs), dim3(256), 0, 0, out, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms;
        (void)hipEventElapsedTime(&ms, e0, e1);
        if (rep && ms < best) best = ms;
      }
      const double flops = (double)wgs * 4 * iters * 256.0 * 512;
      printf("%s operands, %d wgs: %.3f ms  %.1f TFLOP/s\n", r ? "random" : "fixed ", wgs, best,
             flops / best / 1e9);
    }
  }
  return 0;
}
