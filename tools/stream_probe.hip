// stream_probe.hip — how fast can one persistent 1024-thread workgroup per CU stream a
// contiguous chunk of a CSR (int32 col + fp64 val) with the load widths the band SpMM uses
// (4 B + 8 B per lane) vs 16 B per lane?  (diagnostic tool)
#include <hip/hip_runtime.h>

#include <cstdio>

// narrow: lane i loads col[i] (dword) and val[i] (dwordx2), 3 entries per lane per "tile"
__global__ __launch_bounds__(1024) void k_narrow(const int* __restrict__ col, const double* __restrict__ val,
                                                 long long per_wg, double* out) {
  const long long b0 = blockIdx.x * per_wg;
  double acc = 0.0;
  for (long long e = b0 + threadIdx.x; e < b0 + per_wg; e += 1024) acc += val[e] * col[e];
  if (acc == 1.2345) out[0] = acc;
}
// wide: lane loads 4 cols (dwordx4) and 2+2 vals (2 x dwordx4)
__global__ __launch_bounds__(1024) void k_wide(const int4* __restrict__ col, const double2* __restrict__ val,
                                               long long per_wg, double* out) {
  const long long b0 = blockIdx.x * per_wg / 4;
  double acc = 0.0;
  for (long long e = b0 + threadIdx.x; e < b0 + per_wg / 4; e += 1024) {
    const int4 c = col[e];
    const double2 v0 = val[2 * e], v1 = val[2 * e + 1];
    acc += v0.x * c.x + v0.y * c.y + v1.x * c.z + v1.y * c.w;
  }
  if (acc == 1.2345) out[0] = acc;
}
// narrow, unrolled x4 (more loads in flight per wave)
__global__ __launch_bounds__(1024) void k_narrow4(const int* __restrict__ col, const double* __restrict__ val,
                                                  long long per_wg, double* out) {
  const long long b0 = blockIdx.x * per_wg;
  double acc = 0.0;
  for (long long e = b0 + threadIdx.x; e + 3 * 1024 < b0 + per_wg; e += 4096) {
    int c[4];
    double v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) { c[u] = col[e + u * 1024]; v[u] = val[e + u * 1024]; }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc += v[u] * c[u];
  }
  if (acc == 1.2345) out[0] = acc;
}

int main() {
  const long long nnz = 1000000000LL;
  int* col;
  double* val;
  double* out;
  if (hipMalloc(&col, nnz * 4) != hipSuccess || hipMalloc(&val, nnz * 8) != hipSuccess) return 1;
  (void)hipMalloc(&out, 64);
  (void)hipMemset(col, 0, nnz * 4);
  (void)hipMemset(val, 0, nnz * 8);
  const int grid = 256;
  const long long per_wg = nnz / grid / 4096 * 4096;
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  for (int k = 0; k < 3; ++k) {
    for (int rep = 0; rep < 2; ++rep) {
      (void)hipEventRecord(e0);
      if (k == 0) hipLaunchKernelGGL(k_narrow, dim3(grid), dim3(1024), 0, 0, col, val, per_wg, out);
      if (k == 1) hipLaunchKernelGGL(k_narrow4, dim3(grid), dim3(1024), 0, 0, col, val, per_wg, out);
      if (k == 2) hipLaunchKernelGGL(k_wide, dim3(grid), dim3(1024), 0, 0, (const int4*)col, (const double2*)val, per_wg, out);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      const double bytes = (double)per_wg * grid * 12;
      if (rep) printf("%-10s %.3f ms  %.2f TB/s\n", k == 0 ? "narrow" : k == 1 ? "narrow x4" : "wide16B", ms, bytes / ms / 1e9);
    }
  }
  return 0;
}
