// Probe of the int8 MFMA on gfx950 (diagnostic tool) — the building block of an
// Ozaki-style fp64 emulation for the partial-reorth GEMMs:
//   1. lane maps of v_mfma_i32_32x32x32_i8 and v_mfma_i32_16x16x64_i8, checked with exact
//      integer data against a host product (asymmetric operands);
//   2. throughput: independent accumulators back to back on every CU (random operands), and
//      the same loop with the VALU work of splitting fp64 values into int8 digits beside it.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/i8_probe tools/i8_probe.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

typedef int i4v __attribute__((ext_vector_type(4)));
typedef int i16v __attribute__((ext_vector_type(16)));

#define HC(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
  std::printf("HIP %s at %d\n", hipGetErrorString(e_), __LINE__); std::exit(1); } } while (0)

// hypothesis (bf16 32x32x16 pattern at 2x K): lane l, r = l & 31, h = l >> 5 holds
// A[r][16h + j] and B[16h + j][r] in byte j = 0..15; D[row (reg&3) + 8(reg>>2) + 4h][col r]
__global__ void k_layout32(const int8_t* A, const int8_t* B, int* D) {
  const int l = threadIdx.x, r = l & 31, h = l >> 5;
  union { i4v v; int8_t b[16]; } a, bb;
  for (int j = 0; j < 16; ++j) {
    a.b[j] = A[r * 32 + 16 * h + j];
    bb.b[j] = B[(16 * h + j) * 32 + r];
  }
  i16v acc = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_32x32x32_i8(a.v, bb.v, acc, 0, 0, 0);
  for (int reg = 0; reg < 16; ++reg) {
    const int row = (reg & 3) + 8 * (reg >> 2) + 4 * h;
    D[row * 32 + r] = acc[reg];
  }
}
// 16x16x64: lane l, r = l & 15, q = l >> 4 holds A[r][16q + j], B[16q + j][r];
// D[row 4q + reg][col r]
__global__ void k_layout16(const int8_t* A, const int8_t* B, int* D) {
  const int l = threadIdx.x, r = l & 15, q = l >> 4;
  union { i4v v; int8_t b[16]; } a, bb;
  for (int j = 0; j < 16; ++j) {
    a.b[j] = A[r * 64 + 16 * q + j];
    bb.b[j] = B[(16 * q + j) * 16 + r];
  }
  i4v acc = {0, 0, 0, 0};
  acc = __builtin_amdgcn_mfma_i32_16x16x64_i8(a.v, bb.v, acc, 0, 0, 0);
  for (int reg = 0; reg < 4; ++reg) D[(4 * q + reg) * 16 + r] = acc[reg];
}

template <int NACC>
__global__ __launch_bounds__(256) void k_rate32(int* out, int iters, int seed) {
  i16v acc[NACC];
  for (int i = 0; i < NACC; ++i)
    for (int j = 0; j < 16; ++j) acc[i][j] = 0;
  i4v a, b;
  for (int j = 0; j < 4; ++j) {
    a[j] = (int)(0x9E3779B9u * (threadIdx.x + 17 * j + seed));
    b[j] = (int)(0x85EBCA6Bu * (threadIdx.x + 31 * j + seed));
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
  }
  int s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

// MFMA loop with the digit split of 16 fp64 values per lane per `per` MFMAs beside it:
// v = x * 2^54 as two int32 words, 8 base-128 digits, packed 4 per register (the operand of
// the next MFMAs) — the VALU cost an Ozaki Gram pays per 32-row chunk
template <int NACC>
__global__ __launch_bounds__(256) void k_rate32_split(int* out, const double* x, int iters,
                                                      int per) {
  i16v acc[NACC];
  for (int i = 0; i < NACC; ++i)
    for (int j = 0; j < 16; ++j) acc[i][j] = 0;
  i4v a = {1, 2, 3, 4}, b = {5, 6, 7, 8};
  const double* xp = x + (threadIdx.x & 63) * 16;
  for (int it = 0; it < iters; ++it) {
    // split 16 values into 8 digit planes (32 registers), fold into the operands
    i4v planes[8];
    for (int p = 0; p < 8; ++p) planes[p] = i4v{0, 0, 0, 0};
#pragma unroll
    for (int e = 0; e < 16; ++e) {
      const double v = xp[e] * (double)(it + 1);
      const double s = v * 0x1p22;  // 2^54 / 2^32: the high word
      const double hi = __builtin_floor(s);
      const int h = (int)hi;
      const unsigned lo = (unsigned)((s - hi) * 0x1p32);
#pragma unroll
      for (int p = 0; p < 8; ++p) {
        // digit p (p = 0 top, signed) of the 56-bit two's complement (h:lo)
        const int sh = 49 - 7 * p;
        int d;
        if (sh >= 32) d = h >> (sh - 32);
        else if (sh + 7 <= 32) d = (int)((lo >> sh) & 127u);
        else d = (int)(((lo >> sh) | ((unsigned)h << (32 - sh))) & 127u);
        if (p > 0) d &= 127;
        planes[p][e >> 2] |= (d & 255) << (8 * (e & 3));
      }
    }
    a ^= planes[it & 7];
    b ^= planes[(it + 3) & 7];
    for (int k = 0; k < per; ++k) {
#pragma unroll
      for (int i = 0; i < NACC; ++i) acc[i] = __builtin_amdgcn_mfma_i32_32x32x32_i8(a, b, acc[i], 0, 0, 0);
    }
  }
  int s = 0;
  for (int i = 0; i < NACC; ++i) s += acc[i][0] + acc[i][15];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  // ---- layouts ----
  {
    std::vector<int8_t> A(32 * 32), B(32 * 32);
    for (int i = 0; i < 32; ++i)
      for (int k = 0; k < 32; ++k) {
        A[i * 32 + k] = (int8_t)((i * 7 + k * 3) % 23 - 11);
        B[k * 32 + i] = (int8_t)((k * 5 + i * 11) % 19 - 9 + (i > k ? 3 : 0));
      }
    int8_t *dA, *dB;
    int* dD;
    HC(hipMalloc(&dA, 1024));
    HC(hipMalloc(&dB, 1024));
    HC(hipMalloc(&dD, 1024 * 4));
    HC(hipMemcpy(dA, A.data(), 1024, hipMemcpyHostToDevice));
    HC(hipMemcpy(dB, B.data(), 1024, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_layout32, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    std::vector<int> D(1024);
    HC(hipMemcpy(D.data(), dD, 4096, hipMemcpyDeviceToHost));
    int bad = 0;
    for (int i = 0; i < 32; ++i)
      for (int j = 0; j < 32; ++j) {
        int ref = 0;
        for (int k = 0; k < 32; ++k) ref += A[i * 32 + k] * B[k * 32 + j];
        bad += ref != D[i * 32 + j];
      }
    std::printf("layout 32x32x32_i8: %d of 1024 wrong\n", bad);
    std::vector<int8_t> A2(16 * 64), B2(64 * 16);
    for (int i = 0; i < 16; ++i)
      for (int k = 0; k < 64; ++k) {
        A2[i * 64 + k] = (int8_t)((i * 7 + k * 3) % 23 - 11);
        B2[k * 16 + i] = (int8_t)((k * 5 + i * 11) % 19 - 9 + (i > (k & 15) ? 3 : 0));
      }
    HC(hipMemcpy(dA, A2.data(), 1024, hipMemcpyHostToDevice));
    HC(hipMemcpy(dB, B2.data(), 1024, hipMemcpyHostToDevice));
    hipLaunchKernelGGL(k_layout16, dim3(1), dim3(64), 0, 0, dA, dB, dD);
    HC(hipMemcpy(D.data(), dD, 256 * 4, hipMemcpyDeviceToHost));
    bad = 0;
    for (int i = 0; i < 16; ++i)
      for (int j = 0; j < 16; ++j) {
        int ref = 0;
        for (int k = 0; k < 64; ++k) ref += A2[i * 64 + k] * B2[k * 16 + j];
        bad += ref != D[i * 16 + j];
      }
    std::printf("layout 16x16x64_i8: %d of 256 wrong\n", bad);
  }
  // ---- rates ----
  int dev = 0, ncu = 0;
  HC(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev));
  int* out;
  HC(hipMalloc(&out, (size_t)ncu * 8 * 256 * 4));
  double* x;
  HC(hipMalloc(&x, 64 * 16 * 8));
  {
    std::vector<double> hx(64 * 16);
    for (size_t i = 0; i < hx.size(); ++i) hx[i] = ((double)(i * 2654435761u % 100003) / 100003.0 - 0.5) * 1e-3;
    HC(hipMemcpy(x, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  HC(hipEventCreate(&e0));
  HC(hipEventCreate(&e1));
  const int iters = 4000;
  for (int wpc : {4, 8}) {  // waves per CU (256-thread blocks = 4 waves)
    const int grid = ncu * wpc / 4;
    hipLaunchKernelGGL(k_rate32<4>, dim3(grid), dim3(256), 0, 0, out, 100, 1);
    HC(hipEventRecord(e0));
    hipLaunchKernelGGL(k_rate32<4>, dim3(grid), dim3(256), 0, 0, out, iters, 1);
    HC(hipEventRecord(e1));
    HC(hipEventSynchronize(e1));
    float ms;
    HC(hipEventElapsedTime(&ms, e0, e1));
    const double ops = (double)grid * 4 * iters * 4 * 32.0 * 32 * 32 * 2;
    std::printf("i8 32x32x32, %d waves/CU: %.1f TOPS (%.3f ms)\n", wpc, ops / (ms * 1e-3) / 1e12, ms);
  }
  for (int per : {1, 2, 4, 9}) {  // MFMAs (x4 accumulators) per 16-value split
    const int grid = ncu * 8 / 4;
    const int it2 = iters / per;
    hipLaunchKernelGGL(k_rate32_split<4>, dim3(grid), dim3(256), 0, 0, out, x, 10, per);
    HC(hipEventRecord(e0));
    hipLaunchKernelGGL(k_rate32_split<4>, dim3(grid), dim3(256), 0, 0, out, x, it2, per);
    HC(hipEventRecord(e1));
    HC(hipEventSynchronize(e1));
    float ms;
    HC(hipEventElapsedTime(&ms, e0, e1));
    const double ops = (double)grid * 4 * it2 * per * 4 * 32.0 * 32 * 32 * 2;
    std::printf("i8 + split (%d x 4 MFMAs per 16-value split), 8 waves/CU: %.1f TOPS (%.3f ms)\n",
                per, ops / (ms * 1e-3) / 1e12, ms);
  }
  HC(hipDeviceSynchronize());
  return 0;
}
