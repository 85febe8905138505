// basis_stream_probe.hip — what HBM rate do the partial-reorth kernels' basis access patterns
// allow without any MFMA work?  (diagnostic)
// The basis: P panels of n rows x 16 doubles (b = 16, C3's n = 1,585,478 by default), read with
//   contig  : k_gram44's split layout — workgroup = (row split, group of 4 panel pairs), each
//             wave sweeps its pair's rows of the split in 16-row chunks, 8-B loads per lane
//   inter   : the same waves and loads, but split s takes chunks s, s + S, s + 2S, ... so the
//             whole chip sweeps each panel front to back together
//   rowtile : k_tsmm44's layout — workgroup = 128 rows, each wave 32 rows of every panel in turn
//   flat    : the basis as one array, grid-stride 16-B loads
// Each pattern sums what it reads (one store per lane, never taken) so nothing is optimised out.
// usage: basis_stream_probe [n] [panels]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

__global__ void k_fill(double* p, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x)
    p[i] = (double)(i & 1023) * 1e-3;
}

// lane: row (lane >> 4) of each 4-row quad, column (lane & 15); 4 quads per 16-row chunk, two
// panels per wave (the pair), as gram44_body's PAIR load_a
template <bool INTER>
__global__ __launch_bounds__(256) void k_contig(const double* __restrict__ W, long long n, long long stride,
                                               int npairs, int npg, int splits, long long rows_per,
                                               double* out) {
  const int bid = blockIdx.x, xcd = bid & 7, t = bid >> 3;
  const int pg = t % npg;
  const long long s = (long long)(t / npg) * 8 + xcd;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int pair = pg * 4 + wave;
  if (pair >= npairs) return;
  const double* p0 = W + (long long)(2 * pair) * stride;
  const double* p1 = p0 + stride;
  const long long nch = n / 16;
  double acc = 0.0;
  if (INTER) {
#pragma unroll 2
    for (long long c = s; c < nch; c += splits) {
      const long long r = c * 16;
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const long long o = (r + 4 * ks + (lane >> 4)) * 16 + (lane & 15);
        acc += p0[o] + p1[o];
      }
    }
  } else {
    const long long r0 = s * rows_per, r1 = r0 + rows_per < n ? r0 + rows_per : n;
#pragma unroll 2
    for (long long r = r0; r + 16 <= r1; r += 16) {
#pragma unroll
      for (int ks = 0; ks < 4; ++ks) {
        const long long o = (r + 4 * ks + (lane >> 4)) * 16 + (lane & 15);
        acc += p0[o] + p1[o];
      }
    }
  }
  if (acc == 1.2345) out[0] = acc;
}

// k_tsmm44 (b = 16): wave rows r0 .. r0 + 32, per chunk of 32 k (two panels) lane loads 16 B
// (k = 8h + 2q .. +1) of rows (lane & 15) and (lane & 15) + 16
__global__ __launch_bounds__(256) void k_rowtile(const double* __restrict__ W, long long n, long long stride,
                                                int panels, double* out) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane >> 4;
  const long long r0 = ((long long)blockIdx.x * 4 + wave) * 32;
  if (r0 + 32 > n) return;
  double acc = 0.0;
#pragma unroll 2
  for (int ch = 0; ch < panels / 2; ++ch) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int k = ch * 32 + 8 * h + 2 * q;
      const double* xp = W + (long long)(k / 16) * stride + (k % 16);
#pragma unroll
      for (int rt = 0; rt < 2; ++rt) {
        const double2 v = *reinterpret_cast<const double2*>(xp + (r0 + 16 * rt + (lane & 15)) * 16);
        acc += v.x + v.y;
      }
    }
  }
  if (acc == 1.2345) out[0] = acc;
}

__global__ __launch_bounds__(256) void k_flat(const double2* __restrict__ W, long long n2, double* out) {
  double acc = 0.0;
#pragma unroll 4
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n2; i += (long long)gridDim.x * 256) {
    const double2 v = W[i];
    acc += v.x + v.y;
  }
  if (acc == 1.2345) out[0] = acc;
}

int main(int argc, char** argv) {
  const long long n = argc > 1 ? atoll(argv[1]) : 1585478;
  const int panels = argc > 2 ? atoi(argv[2]) : 72;
  const long long stride = n * 16;
  const double bytes = 8.0 * stride * panels;
  double *W, *out;
  if (hipMalloc(&W, (size_t)(8.0 * stride * panels)) != hipSuccess) return 1;
  (void)hipMalloc(&out, 64);
  hipLaunchKernelGGL(k_fill, dim3(8192), dim3(256), 0, 0, W, stride * panels);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int npairs = panels / 2, npg = (npairs + 3) / 4;
  auto timeit = [&](const char* name, auto launch) {
    float best = 1e30f;
    for (int rep = 0; rep < 5; ++rep) {
      (void)hipEventRecord(e0);
      launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (rep && ms < best) best = ms;
    }
    printf("%-28s %8.3f ms  %6.2f TB/s\n", name, best, bytes / best / 1e9);
  };
  for (int splits : {768, 1024, 2048}) {
    long long rows_per = (n + splits - 1) / splits;
    rows_per = (rows_per + 15) / 16 * 16;
    char nm[64];
    snprintf(nm, sizeof nm, "contig splits=%d", splits);
    timeit(nm, [&] { hipLaunchKernelGGL(k_contig<false>, dim3(npg * splits), dim3(256), 0, 0, W, n, stride, npairs, npg, splits, rows_per, out); });
    snprintf(nm, sizeof nm, "inter  splits=%d", splits);
    timeit(nm, [&] { hipLaunchKernelGGL(k_contig<true>, dim3(npg * splits), dim3(256), 0, 0, W, n, stride, npairs, npg, splits, rows_per, out); });
  }
  timeit("rowtile (128 rows per WG)", [&] { hipLaunchKernelGGL(k_rowtile, dim3((unsigned)((n + 127) / 128)), dim3(256), 0, 0, W, n, stride, panels, out); });
  timeit("flat grid-stride 16 B", [&] { hipLaunchKernelGGL(k_flat, dim3(4096), dim3(256), 0, 0, (const double2*)W, stride * panels / 2, out); });
  return 0;
}
