// reorth_probe.cpp — time the shipped partial-reorth kernels (gram44_partial + reduce_slab,
// tsmm44) at n = 1e7, b = 32, X = [Q_i, Q_{i-1}] for a range of basis sizes (diagnostic).
// Build: tools/build_probe.sh (links the library's objects).
#include <hip/hip_runtime.h>

#include <cstdio>
#include <algorithm>
#include <cstdlib>
#include <vector>

#include "../gpu-randomized-block-lanczos_amd/csrc/kernels.hpp"

__global__ void k_fill(double* p, int64_t n, uint64_t seed) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t z = (uint64_t)i * 0x9E3779B97F4A7C15ull + seed;
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z ^= z >> 31;
    p[i] = ((double)(z >> 11) * 0x1.0p-53 - 0.5) * 1e-2;
  }
}
static void fill(double* p, int64_t n, uint64_t seed) {
  hipLaunchKernelGGL(k_fill, dim3(4096), dim3(256), 0, 0, p, n, seed);
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atoll(argv[1]) : 10000000;
  // argv: n, b (32 or 16), nWmax (default 36; C3 at b = 16: 1585478 16 72)
  const int b = argc > 2 ? atoi(argv[2]) : 32, nWmax = argc > 3 ? atoi(argv[3]) : 36;
  const int xw = 2 * b;  // X = [Q_i, Q_{i-1}] columns
  double *W, *X0, *X1, *slab, *C, *Cg;
  if (hipMalloc(&W, (size_t)n * b * nWmax * 8) != hipSuccess) return 1;
  (void)hipMalloc(&X0, (size_t)n * b * 8);
  (void)hipMalloc(&X1, (size_t)n * b * 8);
  fill(W, n * b * nWmax, 1);
  fill(X0, n * b, 2);
  fill(X1, n * b, 3);
  size_t slab_elems = 0;  // the split count may depend on nW: size for the largest product
  for (int nW = 2; nW <= nWmax; nW += 2)
    slab_elems = std::max(slab_elems, (size_t)rbl::gram44_splits(n, nW, b) * nW * b * xw);
  (void)hipMalloc(&slab, slab_elems * 8);
  (void)hipMalloc(&C, (size_t)nWmax * b * xw * 8);
  fill(C, nWmax * b * xw, 4);
  (void)hipMalloc(&Cg, (size_t)nWmax * b * xw * 8);
  // PROBE_XG=1: the update also forms Q_{i-1}^T Q_i (the fused local-reorth Gram)
  const bool xg = getenv("PROBE_XG") && atoi(getenv("PROBE_XG"));
  double* xslab = nullptr;
  int xgrid = 0;
  if (hipMalloc(&xslab, (size_t)rbl::tsmm44_xg_grid(n) * 1024 * 8) != hipSuccess) return 1;
  hipEvent_t e0, e1, e2;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventCreate(&e2);
  double tg = 0, tt = 0, fl = 0, byg = 0, byt = 0;
  for (int nW = 2; nW <= nWmax; nW += 2) {
    rbl::PanelRun Wr;
    Wr.base = W;
    // PROBE_W0=1: every panel aliases panel 0 (same instruction stream and MFMAs, the basis
    // served from L2 / Infinity Cache instead of HBM) — separates data movement from MFMA issue
    Wr.stride = (getenv("PROBE_W0") && atoi(getenv("PROBE_W0"))) ? 0 : n * b;
    Wr.count = nW;
    Wr.w = b;
    rbl::Panels X;
    X.ptr[0] = X0;
    X.ptr[1] = X1;
    X.count = 2;
    X.w = b;
    const int splits = rbl::gram44_splits(n, nW, b);
    float bg = 1e30f, bt = 1e30f;
    for (int rep = 0; rep < 3; ++rep) {
      (void)hipEventRecord(e0);
      rbl::gram44_partial(n, Wr, X, slab, splits, nullptr, 0);
      rbl::reduce_slab(slab, splits, (int64_t)nW * b * xw, Cg, nullptr, 0);  // C stays fixed: X must not blow up
      (void)hipEventRecord(e1);
      rbl::tsmm44(n, Wr, C, xw, X, -1.0, 1.0, nullptr, 0, xg ? xslab : nullptr, &xgrid);
      (void)hipEventRecord(e2);
      (void)hipEventSynchronize(e2);
      float g, t;
      (void)hipEventElapsedTime(&g, e0, e1);
      (void)hipEventElapsedTime(&t, e1, e2);
      if (rep) {
        bg = g < bg ? g : bg;
        bt = t < bt ? t : bt;
      }
    }
    const double f = 2.0 * n * nW * b * xw;
    printf("nW=%2d  splits %4d  gram %7.3f ms %5.1f TF   tsmm %7.3f ms %5.1f TF\n", nW, splits, bg, f / bg / 1e9, bt,
           f / bt / 1e9);
    byg += 8.0 * n * (nW * b + xw);       // basis + X read once
    byt += 8.0 * n * (nW * b + 2 * xw);   // basis read, X read and written
    tg += bg;
    tt += bt;
    fl += f;
  }
  printf("sum over nW=2..%d step 2: gram %.1f ms (%.1f TF, %.2f TB/s)  tsmm %.1f ms (%.1f TF, %.2f TB/s)\n", nWmax,
         tg, fl / tg / 1e9, byg / tg / 1e9, tt, fl / tt / 1e9, byt / tt / 1e9);
  return 0;
}
