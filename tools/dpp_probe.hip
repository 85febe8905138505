// Probe of gfx950 DPP row_newbcast semantics used by spmm_window.hip (diagnostic tool).
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void k(const double* x, const double* y, const unsigned* o, double* r1, unsigned* r2, double* r3) {
  int l = threadIdx.x;
  double v = x[l], q = y[l], acc = 0.0;
  unsigned off = o[l], lo = 1000u * (l & 15), ad;
  asm volatile("s_nop 1" : "+v"(v), "+v"(off));
  asm volatile("v_fmac_f64_dpp %0, %1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(v), "v"(q));
  asm volatile("v_add_u32_dpp %0, %1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf" : "=v"(ad) : "v"(off), "v"(lo));
  r1[l] = acc; r2[l] = ad;
  double m;
  asm volatile("v_mov_b64_dpp %0, %1 row_newbcast:7 row_mask:0xf bank_mask:0xf" : "=v"(m) : "v"(v));
  r3[l] = m;
}
int main() {
  double hx[64], hy[64]; unsigned ho[64];
  for (int i = 0; i < 64; ++i) { hx[i] = 100 + i; hy[i] = 1.0 + 0.001 * i; ho[i] = 10 * i; }
  double *x, *y, *r1, *r3; unsigned *o, *r2;
  hipMalloc(&x, 512); hipMalloc(&y, 512); hipMalloc(&o, 256); hipMalloc(&r1, 512); hipMalloc(&r2, 256); hipMalloc(&r3, 512);
  hipMemcpy(x, hx, 512, hipMemcpyHostToDevice); hipMemcpy(y, hy, 512, hipMemcpyHostToDevice); hipMemcpy(o, ho, 256, hipMemcpyHostToDevice);
  hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, x, y, o, r1, r2, r3);
  double h1[64], h3[64]; unsigned h2[64];
  hipMemcpy(h1, r1, 512, hipMemcpyDeviceToHost); hipMemcpy(h2, r2, 256, hipMemcpyDeviceToHost); hipMemcpy(h3, r3, 512, hipMemcpyDeviceToHost);
  int bad = 0;
  for (int l = 0; l < 64; ++l) {
    int row = l >> 4;
    double e1 = hx[row * 16 + 3] * hy[l];
    unsigned e2 = ho[row * 16 + 5] + 1000u * (l & 15);
    double e3 = hx[row * 16 + 7];
    if (h1[l] != e1 || h2[l] != e2 || h3[l] != e3) { ++bad; if (bad < 8) printf("lane %d: fmac %g (exp %g) add %u (exp %u) mov64 %g (exp %g)\n", l, h1[l], e1, h2[l], e2, h3[l], e3); }
  }
  printf("dpp probe: %d bad lanes\n", bad);
  return bad != 0;
}
