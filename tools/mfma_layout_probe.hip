// Infers the lane layout of v_mfma_f64_4x4x4f64 (diagnostic tool): for A = e_p (one lane set),
// B[l] = l + 1, the nonzero outputs D[l] = B[lane holding (k_p, col(l))] reveal the map.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(double* D) {
  int l = threadIdx.x;
  for (int p = 0; p < 64; ++p) {
    double a = (l == p) ? 1.0 : 0.0, b = l + 1.0;
    double d = __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, 0.0, 0, 0, 0);
    D[p * 64 + l] = d;
  }
}
int main() {
  double* d; (void)hipMalloc(&d, 64 * 64 * 8);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, d);
  double h[64 * 64]; (void)hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
  for (int p = 0; p < 64; ++p) {
    printf("A-lane %2d ->", p);
    for (int l = 0; l < 64; ++l) if (h[p * 64 + l] != 0) printf(" D%d=B%d", l, (int)h[p * 64 + l] - 1);
    printf("\n");
  }
  return 0;
}
