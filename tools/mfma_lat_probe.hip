// mfma_lat_probe.hip — v_mfma_f64_4x4x4f64 dependent-chain latency vs independent
// accumulators, and LDS read latency in front of an MFMA (diagnostic tool).
// Cycles from s_memtime (shader clock) around the loop, one wave per SIMD and four.
#include <hip/hip_runtime.h>

#include <cstdio>

template <int NACC>
__global__ void k_chain(double* out, long long* cyc, int iters, double a0) {
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = 0.0;
  const double a = a0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

// one LDS read feeding each MFMA of a single chain (the band-kernel pattern)
__global__ void k_lds_chain(double* out, long long* cyc, int iters) {
  __shared__ double buf[4096];
  for (int i = threadIdx.x; i < 4096; i += blockDim.x) buf[i] = 1.0 + i * 1e-6;
  __syncthreads();
  double acc = 0.0;
  const double a = 1.0 + threadIdx.x * 1e-3;
  int idx = threadIdx.x;
  const long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    const double b = buf[idx];
    acc = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc, 0, 0, 0);
    idx = (idx + 64) & 4095;
  }
  const long long t1 = __builtin_amdgcn_s_memtime();
  out[blockIdx.x * blockDim.x + threadIdx.x] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <typename F>
static void run(const char* name, F launch, int blocks, int iters, int per_iter) {
  long long* cyc;
  (void)hipMalloc(&cyc, blocks * sizeof(long long));
  launch(cyc);
  (void)hipDeviceSynchronize();
  long long h[4];
  (void)hipMemcpy(h, cyc, sizeof(h), hipMemcpyDeviceToHost);
  printf("%-34s blocks=%5d  %.2f cycles per MFMA issue per wave\n", name, blocks,
         (double)h[0] / ((double)iters * per_iter));
  (void)hipFree(cyc);
}

int main() {
  double* out;
  (void)hipMalloc(&out, 1 << 26);
  const int iters = 4096;
  for (int blocks : {256 * 4, 256 * 16}) {  // 1 and 4 waves per SIMD (64-thread blocks)
    run("chain x1", [&](long long* c) { hipLaunchKernelGGL(k_chain<1>, dim3(blocks), dim3(64), 0, 0, out, c, iters, 0.5); }, blocks, iters, 1);
    run("chain x2", [&](long long* c) { hipLaunchKernelGGL(k_chain<2>, dim3(blocks), dim3(64), 0, 0, out, c, iters, 0.5); }, blocks, iters, 2);
    run("chain x4", [&](long long* c) { hipLaunchKernelGGL(k_chain<4>, dim3(blocks), dim3(64), 0, 0, out, c, iters, 0.5); }, blocks, iters, 4);
    run("chain x8", [&](long long* c) { hipLaunchKernelGGL(k_chain<8>, dim3(blocks), dim3(64), 0, 0, out, c, iters, 0.5); }, blocks, iters, 8);
    run("lds->mfma chain", [&](long long* c) { hipLaunchKernelGGL(k_lds_chain, dim3(blocks), dim3(64), 0, 0, out, c, iters); }, blocks, iters, 1);
  }
  return 0;
}
