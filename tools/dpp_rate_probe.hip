// Throughput of the instructions in the LDS-window SpMM inner loop (diagnostic tool):
// v_fmac_f64 vs v_fmac_f64_dpp row_newbcast, v_add_u32 vs v_add_u32_dpp, ds_read_b128.
#include <hip/hip_runtime.h>
#include <cstdio>

template <int MODE>
__global__ __launch_bounds__(256) void k(double* out, int iters) {
  double acc[16];
  for (int i = 0; i < 16; ++i) acc[i] = threadIdx.x + i;
  double v = 1.0 + threadIdx.x * 1e-6, q = 0.999;
  unsigned o = threadIdx.x, lo = 4 * threadIdx.x, r = 0;
  asm volatile("s_nop 4" : "+v"(v), "+v"(o));
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      if constexpr (MODE == 0) asm volatile("v_fmac_f64_e32 %0, %1, %2" : "+v"(acc[i]) : "v"(v), "v"(q));
      if constexpr (MODE == 1)
        asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(acc[i]) : "v"(v), "v"(q));
      if constexpr (MODE == 2) { unsigned t; asm volatile("v_add_u32_e32 %0, %1, %2" : "=v"(t) : "v"(o), "v"(lo)); r += t; }
      if constexpr (MODE == 3) {
        unsigned t;
        asm volatile("v_add_u32_dpp %0, %1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf" : "=v"(t) : "v"(o), "v"(lo));
        r ^= t;
      }
    }
  }
  double s = r;
  for (int i = 0; i < 16; ++i) s += acc[i];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

// ds_read_b128 of 256-B ring rows: 4 lane groups read 4 rows, 16 B per lane
__global__ __launch_bounds__(1024) void k_lds(double* out, int iters) {
  __shared__ __attribute__((aligned(16))) double ring[256 * 32];
  for (int i = threadIdx.x; i < 256 * 32; i += 1024) ring[i] = i;
  __syncthreads();
  typedef double d2 __attribute__((ext_vector_type(2)));
  const int lane = threadIdx.x & 63, g = lane >> 4, li = lane & 15;
  unsigned row = (threadIdx.x * 7 + g * 13) & 255;
  double s0 = 0, s1 = 0;
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const d2 v = *(const d2*)&ring[((row + i * 37) & 255) * 32 + li * 2];
      s0 += v[0];
      s1 += v[1];
    }
    row = (row + 11) & 255;
  }
  out[blockIdx.x * 1024 + threadIdx.x] = s0 + s1;
}

int main() {
  double* out;
  (void)hipMalloc(&out, 1 << 26);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int wgs = 2048, iters = 4000;
  const char* names[4] = {"v_fmac_f64", "v_fmac_f64_dpp", "v_add_u32", "v_add_u32_dpp"};
  for (int m = 0; m < 4; ++m) {
    float ms;
    auto run = [&](int it) {
      switch (m) {
        case 0: hipLaunchKernelGGL(k<0>, dim3(wgs), dim3(256), 0, 0, out, it); break;
        case 1: hipLaunchKernelGGL(k<1>, dim3(wgs), dim3(256), 0, 0, out, it); break;
        case 2: hipLaunchKernelGGL(k<2>, dim3(wgs), dim3(256), 0, 0, out, it); break;
        default: hipLaunchKernelGGL(k<3>, dim3(wgs), dim3(256), 0, 0, out, it); break;
      }
    };
    run(10);
    (void)hipEventRecord(e0);
    run(iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double winstr = (double)wgs * 4 * iters * 16;  // wave instructions
    // cycles per wave-instruction per SIMD at an assumed 2.4 GHz: SIMD-seconds / instr
    printf("%-16s %.3f G wave-instr/s  -> %.2f SIMD-cycles each @2.4GHz\n", names[m],
           winstr / ms / 1e6, 1024.0 * 2.4e9 / (winstr / ms * 1e3));
  }
  {
    float ms;
    hipLaunchKernelGGL(k_lds, dim3(256), dim3(1024), 0, 0, out, 10);
    (void)hipEventRecord(e0);
    hipLaunchKernelGGL(k_lds, dim3(256), dim3(1024), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double winstr = 256.0 * 16 * iters * 8;
    printf("ds_read_b128 ring rows: %.3f G wave-instr/s -> %.2f CU-cycles each @2.4GHz (%.1f B/clk/CU)\n",
           winstr / ms / 1e6, 256.0 * 2.4e9 / (winstr / ms * 1e3),
           1024.0 / (256.0 * 2.4e9 / (winstr / ms * 1e3)));
  }
  return 0;
}
