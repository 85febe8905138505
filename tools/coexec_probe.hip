// coexec_probe.hip — do fp64 VALU FMAs and fp64 MFMAs (v_mfma_f64_4x4x4f64) execute
// concurrently on gfx950?  Waves of one workgroup split by role: MFMA-only, VALU-only, or
// both in one workgroup (half the waves each).  TFLOP/s per configuration (diagnostic tool).
#include <hip/hip_runtime.h>

#include <cstdio>

template <int MODE>  // 0: all waves MFMA, 1: all waves VALU, 2: even waves MFMA / odd VALU,
                     // 3: all waves int VALU, 4: even waves MFMA / odd int VALU
__global__ __launch_bounds__(512) void k_mix(double* out, int iters, double a0) {
  const int wave = threadIdx.x >> 6;
  const bool mfma = MODE == 0 || ((MODE == 2 || MODE == 4) && (wave & 1) == 0);
  const bool ivalu = MODE == 3 || (MODE == 4 && (wave & 1));
  double acc[8];
  for (int i = 0; i < 8; ++i) acc[i] = i * 1e-3;
  const double a = a0 + threadIdx.x * 1e-6, b = 1.0 - threadIdx.x * 1e-7;
  if (ivalu) {
    unsigned u[8];
    for (int i = 0; i < 8; ++i) u[i] = threadIdx.x * 2654435761u + i;
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) u[i] = (u[i] ^ (u[i] >> 7)) + 0x9E3779B9u;
    }
    for (int i = 0; i < 8; ++i) acc[i] = u[i];
  } else if (mfma) {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
    }
  } else {
    for (int it = 0; it < iters; ++it) {
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] = fma(a, acc[i], b);
    }
  }
  double s = 0;
  for (int i = 0; i < 8; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  double* out;
  (void)hipMalloc(&out, 1 << 26);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int wgs = 256 * 4, iters = 4000;
  for (int mode = 0; mode < 5; ++mode) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(k_mix<0>, dim3(wgs), dim3(512), 0, 0, out, iters, 0.5);
      if (mode == 1) hipLaunchKernelGGL(k_mix<1>, dim3(wgs), dim3(512), 0, 0, out, iters, 0.5);
      if (mode == 2) hipLaunchKernelGGL(k_mix<2>, dim3(wgs), dim3(512), 0, 0, out, iters, 0.5);
      if (mode == 3) hipLaunchKernelGGL(k_mix<3>, dim3(wgs), dim3(512), 0, 0, out, iters, 0.5);
      if (mode == 4) hipLaunchKernelGGL(k_mix<4>, dim3(wgs), dim3(512), 0, 0, out, iters, 0.5);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      // MFMA wave: iters * 8 * 512 flops; VALU wave: iters * 32 * 64 lanes * 2 flops
      const double waves = (double)wgs * 8;
      const double fm = iters * 8.0 * 512, fv = iters * 32.0 * 128;
      double flops = 0;
      if (mode == 0) flops = waves * fm;
      if (mode == 1) flops = waves * fv;
      if (mode == 2) flops = waves / 2 * (fm + fv);
      // int VALU: 2 ops (xor-shift, add) x 32 per iteration, counted as "flops" for the rate
      if (mode == 3) flops = waves * fv;
      if (mode == 4) flops = waves / 2 * (fm + fv);
      static const char* nm[] = {"MFMA only", "fp64 VALU only", "MFMA / fp64 VALU", "int VALU only", "MFMA / int VALU"};
      if (rep) printf("mode %d (%s): %.3f ms  %.1f T(FL)OP/s\n", mode, nm[mode], ms, flops / ms / 1e9);
    }
  }
  return 0;
}
