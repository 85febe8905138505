// PCIe copy rates for the host-spill basis: 2.56 GB (one C4 Krylov block) H2D / D2H with
// pinned host memory (default = coherent, and non-coherent), on an idle GPU and beside a
// streaming kernel.  Build: hipcc -O3 --offload-arch=gfx950 tools/pcie_probe.hip -o tools/pcie_probe
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>

__global__ void k_stream(const double* __restrict__ a, double* __restrict__ b, size_t n, int reps) {
  for (int r = 0; r < reps; ++r)
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
      b[i] = a[i] * 1.0000001 + r;
}

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main() {
  const size_t bytes = 2560ull << 20;
  double *d, *d2, *d3;
  hipMalloc(&d, bytes);
  hipMalloc(&d2, bytes);
  hipMalloc(&d3, bytes);
  hipMemset(d, 0, bytes);
  hipStream_t s1, s2;
  hipStreamCreateWithFlags(&s1, hipStreamNonBlocking);
  hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  for (unsigned flags : {(unsigned)hipHostMallocDefault, (unsigned)hipHostMallocNonCoherent}) {
    double* h;
    hipHostMalloc(&h, bytes, flags);
    for (int busy = 0; busy < 2; ++busy) {
      for (int dir = 0; dir < 2; ++dir) {
        hipDeviceSynchronize();
        if (busy) hipLaunchKernelGGL(k_stream, dim3(2048), dim3(256), 0, s2, d2, d3, bytes / 8, 20);
        const double t0 = now();
        if (dir == 0) hipMemcpyAsync(d, h, bytes, hipMemcpyHostToDevice, s1);
        else hipMemcpyAsync(h, d, bytes, hipMemcpyDeviceToHost, s1);
        hipStreamSynchronize(s1);
        const double t = now() - t0;
        hipDeviceSynchronize();
        printf("pinned %-12s %s %-4s %.1f GB/s\n", flags ? "noncoherent" : "default",
               busy ? "busy" : "idle", dir ? "D2H" : "H2D", bytes / t / 1e9);
      }
    }
    hipHostFree(h);
  }
  return 0;
}
