// Microbenchmark of the ceilings the RBL kernels are priced against (diagnostic tool):
//   * v_mfma_f64_16x16x4f64 throughput (independent accumulators, operands in registers)
//   * streaming HBM read bandwidth (16 B / lane loads) and copy bandwidth
#include <hip/hip_runtime.h>
#include <cstdio>
typedef double d4 __attribute__((ext_vector_type(4)));

template <int NACC>
__global__ __launch_bounds__(256) void k_mfma(double* out, int iters, double a0) {
  d4 acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4{0, 0, 0, 0};
  double a = a0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, acc[i], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

typedef double d4x __attribute__((ext_vector_type(4)));
template <int NACC>
__global__ __launch_bounds__(256) void k_mfma4(double* out, int iters, double a0) {
  d4x acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = d4x{0, 0, 0, 0};
  double a = a0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i][0] = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, acc[i][0], 0, 0, 0);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int NACC>
__global__ __launch_bounds__(256) void k_valu(double* out, int iters, double a0) {
  double acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = i;
  double a = a0 + threadIdx.x * 1e-3, b = 1.0 - threadIdx.x * 1e-4;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = fma(a, acc[i], b);
  }
  double s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
typedef float f4p __attribute__((ext_vector_type(4)));
typedef float f16p __attribute__((ext_vector_type(16)));
template <int NACC>
__global__ __launch_bounds__(256) void k_mfma32(double* out, int iters, float a0) {
  f4p acc[NACC];
  for (int i = 0; i < NACC; ++i) acc[i] = f4p{0, 0, 0, 0};
  float a = a0 + threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][1] + acc[i][2] + acc[i][3];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
template <int NACC>
__global__ __launch_bounds__(256) void k_mfma32x(double* out, int iters, float a0) {
  f16p acc[NACC];
  for (int i = 0; i < NACC; ++i)
    for (int r = 0; r < 16; ++r) acc[i][r] = 0.f;
  float a = a0 + threadIdx.x * 1e-3f, b = 1.0f - threadIdx.x * 1e-4f;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[i], 0, 0, 0);
  }
  float s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}
__global__ void k_read(const double2* __restrict__ x, size_t n2, double* out) {
  double s = 0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) {
    double2 v = x[i];
    s += v.x + v.y;
  }
  if (s == 123.456) out[0] = s;
}
__global__ void k_copy(const double2* __restrict__ x, double2* __restrict__ y, size_t n2) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n2; i += (size_t)gridDim.x * blockDim.x) y[i] = x[i];
}

int main() {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  double* out;
  (void)hipMalloc(&out, 1 << 24);
  float ms;
  for (int wgs : {1024, 2048}) {
    const int iters = 2000;
    hipLaunchKernelGGL(k_mfma<8>, dim3(wgs), dim3(256), 0, 0, out, 10, 0.5);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_mfma<8>, dim3(wgs), dim3(256), 0, 0, out, iters, 0.5);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double flops = (double)wgs * 4 * iters * 8 * 2048.0;
    printf("mfma_f64_16x16x4: %d WGs x 4 waves, 8 acc: %.2f TFLOP/s  (%.3f ms)\n", wgs, flops / ms / 1e9, ms);
  }
  {
    const int wgs = 2048, iters = 2000;
    hipLaunchKernelGGL(k_mfma4<8>, dim3(wgs), dim3(256), 0, 0, out, 10, 0.5);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_mfma4<8>, dim3(wgs), dim3(256), 0, 0, out, iters, 0.5);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("mfma_f64_4x4x4: %.2f TFLOP/s\n", (double)wgs * 4 * iters * 8 * 512.0 / ms / 1e9);
    hipLaunchKernelGGL(k_valu<16>, dim3(wgs), dim3(256), 0, 0, out, 10, 0.5);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_valu<16>, dim3(wgs), dim3(256), 0, 0, out, iters, 0.5);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("valu v_fma_f64: %.2f TFLOP/s\n", (double)wgs * 256 * iters * 16 * 2.0 / ms / 1e9);
  }
  {
    const int wgs = 2048, iters = 2000;
    hipLaunchKernelGGL(k_mfma32<8>, dim3(wgs), dim3(256), 0, 0, out, 10, 0.5f);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_mfma32<8>, dim3(wgs), dim3(256), 0, 0, out, iters, 0.5f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("mfma_f32_16x16x4: %.2f TFLOP/s\n", (double)wgs * 4 * iters * 8 * 2048.0 / ms / 1e9);
    hipLaunchKernelGGL(k_mfma32x<4>, dim3(wgs), dim3(256), 0, 0, out, 10, 0.5f);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_mfma32x<4>, dim3(wgs), dim3(256), 0, 0, out, iters, 0.5f);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("mfma_f32_32x32x2: %.2f TFLOP/s\n", (double)wgs * 4 * iters * 4 * 4096.0 / ms / 1e9);
  }
  const size_t bytes = 8ull << 30;
  double2 *x, *y;
  (void)hipMalloc(&x, bytes);
  (void)hipMalloc(&y, bytes);
  (void)hipMemset(x, 0, bytes);
  (void)hipMemset(y, 0, bytes);
  const size_t n2 = bytes / 16;
  for (int grid : {2048, 4096, 8192}) {
    hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, x, n2, out);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_read, dim3(grid), dim3(256), 0, 0, x, n2, out);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("read  grid %5d: %.1f GB/s\n", grid, 3.0 * bytes / ms / 1e6);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 3; ++r) hipLaunchKernelGGL(k_copy, dim3(grid), dim3(256), 0, 0, x, y, n2);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    printf("copy  grid %5d: %.1f GB/s (read+write)\n", grid, 3.0 * 2 * bytes / ms / 1e6);
  }
  return 0;
}
