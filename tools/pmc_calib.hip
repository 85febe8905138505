// pmc_calib.hip — calibrate rocprofv3 FETCH_SIZE / WRITE_SIZE on gfx950 per access width.
//
// Streams a known byte count (2 GiB, far beyond the 256 MiB Infinity Cache) with 4, 8 and
// 16 B per lane coalesced loads, and writes 2 GiB with 8 B and 16 B stores.  Profile with
//   rocprofv3 --pmc FETCH_SIZE --output-format csv -d <dir> -- ./pmc_calib
//   rocprofv3 --pmc WRITE_SIZE --output-format csv -d <dir> -- ./pmc_calib
// and divide the counter (KB) by the bytes below to get the per-width factor.
#include <hip/hip_runtime.h>

#include <cstdio>

template <typename T>
__global__ void k_read(const T* __restrict__ p, size_t n, double* out) {
  double acc = 0.0;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    const T v = p[i];
    if constexpr (sizeof(T) == 16) {
      acc += (double)v.x + (double)v.y;
    } else {
      acc += (double)v;
    }
  }
  if (acc == 1234.5) out[0] = acc;  // keep the loads alive
}

template <typename T>
__global__ void k_write(T* __restrict__ p, size_t n) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
       i += (size_t)gridDim.x * blockDim.x) {
    if constexpr (sizeof(T) == 16) {
      p[i] = T{(double)i, 1.0};
    } else {
      p[i] = (T)i;
    }
  }
}

int main() {
  const size_t bytes = size_t(2) << 30;
  void* buf = nullptr;
  double* out = nullptr;
  if (hipMalloc(&buf, bytes) != hipSuccess || hipMalloc(&out, 8) != hipSuccess) return 1;
  (void)hipMemset(buf, 0, bytes);
  const dim3 grid(256 * 8 * 4), block(256);
  hipLaunchKernelGGL(k_read<int>, grid, block, 0, 0, (const int*)buf, bytes / 4, out);
  hipLaunchKernelGGL(k_read<double>, grid, block, 0, 0, (const double*)buf, bytes / 8, out);
  hipLaunchKernelGGL(k_read<double2>, grid, block, 0, 0, (const double2*)buf, bytes / 16, out);
  hipLaunchKernelGGL(k_write<double>, grid, block, 0, 0, (double*)buf, bytes / 8);
  hipLaunchKernelGGL(k_write<double2>, grid, block, 0, 0, (double2*)buf, bytes / 16);
  if (hipDeviceSynchronize() != hipSuccess) return 2;
  printf("bytes per kernel: %zu\n", bytes);
  (void)hipFree(buf);
  (void)hipFree(out);
  return 0;
}
