// gen_rmat.hip — device generator of the seeded symmetric R-MAT matrix (SURVEY.md §8(d) C4b,
// BASELINE config 4: n = 1e7, ~1e9 nonzeros, power-law degrees), row slice [r0, r1) per rank.
//
// Definition (restated in NumPy by oracle/matgen.py: rmat_csr; bit-exact):
//   edge draw e = 0..E-1 descends `scale` levels; level l draws u = u53(pair_hash(seed ^ kRmatK,
//   e, l)) and takes quadrant (0,0) if u < a, (0,1) if u < a+b, (1,0) if u < a+b+c, else (1,1),
//   setting bit (scale-1-l) of the row / column id.  Draws with an id >= n or a self loop are
//   dropped; the rest enter as (r,c) and (c,r), duplicates merged.  Off-diagonal values are the
//   hash-window values 2u-1, u = u53(mix64(pair_hash(seed, lo, hi) ^ K)) (so a duplicate pair has
//   one value); every diagonal entry exists with hw_value(seed, r, r) plus the planted spectrum
//   at rows l * floor(n / nplant).
//
// Pipeline: degree histogram (all draws; it balances the row split over ranks by nonzeros),
// keys (row - r0) << 32 | col appended for the own rows, 64-bit radix sort + unique (hipCUB),
// row pointers from the sorted keys (every row has its diagonal), values from the hash.
#include <hipcub/hipcub.hpp>

#include "kernels.hpp"

namespace rbl {

namespace {
constexpr uint64_t kRmatK = 0xD1B54A32D192ED03ull;

__device__ inline void rmat_draw(const RmatParams& p, int64_t e, int64_t* r, int64_t* c) {
  const uint64_t s2 = p.seed ^ kRmatK;
  const double ab = p.a + p.b, abc = ab + p.c;
  int64_t rr = 0, cc = 0;
  for (int l = 0; l < p.scale; ++l) {
    const double u = u53(pair_hash(s2, e, l));
    const int64_t bit = (int64_t)1 << (p.scale - 1 - l);
    if (u >= ab) rr |= bit;                                // (1,0), (1,1)
    if ((u >= p.a && u < ab) || u >= abc) cc |= bit;       // (0,1), (1,1)
  }
  *r = rr;
  *c = cc;
}

// vertex id -> stored row / column id (RBL_OPT_RELABEL: P A P^T)
__device__ inline int64_t rmat_id(const RmatParams& p, int64_t v) {
  return p.relabel ? scatter(p.perm, v) : v;
}

__global__ void k_rmat_degree(RmatParams p, int32_t* __restrict__ deg) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < p.edges; e += stride) {
    int64_t r, c;
    rmat_draw(p, e, &r, &c);
    if (r < p.n && c < p.n && r != c) {
      atomicAdd(deg + rmat_id(p, r), 1);
      atomicAdd(deg + rmat_id(p, c), 1);
    }
  }
}

// keys of the own rows [r0, r1): both orientations of every kept draw, then the diagonal
__global__ void k_rmat_keys(RmatParams p, int64_t r0, int64_t r1, uint64_t* __restrict__ keys,
                            unsigned long long* __restrict__ count) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < p.edges; e += stride) {
    int64_t r, c;
    rmat_draw(p, e, &r, &c);
    if (r >= p.n || c >= p.n || r == c) continue;
    r = rmat_id(p, r);
    c = rmat_id(p, c);
    if (r >= r0 && r < r1) keys[atomicAdd(count, 1ull)] = ((uint64_t)(r - r0) << 32) | (uint64_t)c;
    if (c >= r0 && c < r1) keys[atomicAdd(count, 1ull)] = ((uint64_t)(c - r0) << 32) | (uint64_t)r;
  }
}

__global__ void k_rmat_diag(int64_t r0, int64_t r1, uint64_t* __restrict__ keys) {
  const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i < r1 - r0) keys[i] = ((uint64_t)i << 32) | (uint64_t)(r0 + i);
}

// rowptr from sorted unique keys: every row owns its diagonal, so rows appear in order with
// no gaps; the first entry of row i sets rowptr[i]
__global__ void k_rmat_csr(const uint64_t* __restrict__ keys, int64_t nnz, int64_t r0, int64_t m,
                           uint64_t seed, int nplant, const double* __restrict__ plant, int64_t n,
                           int64_t* __restrict__ rowptr, int32_t* __restrict__ col,
                           double* __restrict__ val, bool relabel, Scatter perm) {
  const int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= nnz) {
    if (k == nnz) rowptr[m] = nnz;
    return;
  }
  const uint64_t key = keys[k];
  const int64_t i = (int64_t)(key >> 32);
  const int64_t c = (int64_t)(key & 0xffffffffull);
  if (k == 0 || (int64_t)(keys[k - 1] >> 32) != i) rowptr[i] = k;
  col[k] = (int32_t)c;
  // values (and the plant) of the original vertex ids
  const int64_t r = relabel ? scatter_inv(perm, r0 + i) : r0 + i;
  const int64_t co = relabel ? scatter_inv(perm, c) : c;
  double v;
  if (co == r) {
    v = hw_value(seed, r, r);
    const int64_t st = nplant > 0 ? n / nplant : 0;
    if (st > 0 && r % st == 0 && r / st < nplant) v += plant[r / st];
  } else {
    v = hw_value(seed, co < r ? co : r, co < r ? r : co);
  }
  val[k] = v;
}

// per-rank column footprint (min, max+1) of the local CSR: block reduction, then one atomic
// per rank per block
__global__ void k_col_footprint(const int32_t* __restrict__ col, int64_t nnz,
                                const int64_t* __restrict__ bounds, int P,
                                unsigned long long* __restrict__ lo, unsigned long long* __restrict__ hi) {
  __shared__ unsigned long long slo[16], shi[16];
  if (threadIdx.x < 16) {
    slo[threadIdx.x] = ~0ull;
    shi[threadIdx.x] = 0ull;
  }
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nnz; e += stride) {
    const int64_t c = col[e];
    int q = 0;
    while (q + 1 < P && c >= bounds[q + 1]) ++q;
    atomicMin(slo + q, (unsigned long long)c);
    atomicMax(shi + q, (unsigned long long)(c + 1));
  }
  __syncthreads();
  if (threadIdx.x < P) {
    if (slo[threadIdx.x] != ~0ull) atomicMin(lo + threadIdx.x, slo[threadIdx.x]);
    if (shi[threadIdx.x] != 0ull) atomicMax(hi + threadIdx.x, shi[threadIdx.x]);
  }
}
}  // namespace

void rmat_degree(const RmatParams& p, int32_t* deg, hipStream_t s) {
  hipLaunchKernelGGL(k_rmat_degree, dim3(4096), dim3(256), 0, s, p, deg);
}

int rmat_local_csr(const RmatParams& p, int64_t r0, int64_t r1, int64_t max_keys, int nplant,
                   const double* plant_dev, int64_t* rowptr_dev, int32_t** col_dev,
                   double** val_dev, int64_t* nnz_out, hipStream_t s) {
  const int64_t m = r1 - r0;
  uint64_t *k0 = nullptr, *k1 = nullptr;
  unsigned long long* d_cnt = nullptr;
  int* d_nsel = nullptr;
  void* tmp = nullptr;
  int rc = 0;
  auto ok = [&](hipError_t e) {
    if (e != hipSuccess && rc == 0) rc = e == hipErrorOutOfMemory ? -3 : -2;
    return rc == 0;
  };
  const int64_t cap = max_keys + m;
  if (cap >= (int64_t)INT32_MAX) return -1;  // hipCUB item counts are int
  if (!ok(hipMalloc(&k0, cap * sizeof(uint64_t))) || !ok(hipMalloc(&k1, cap * sizeof(uint64_t))) ||
      !ok(hipMalloc(&d_cnt, sizeof(unsigned long long))) || !ok(hipMalloc(&d_nsel, sizeof(int)))) {
    hipFree(k0); hipFree(k1); hipFree(d_cnt); hipFree(d_nsel);
    return rc;
  }
  unsigned long long h_cnt = (unsigned long long)m;
  ok(hipMemcpyAsync(d_cnt, &h_cnt, sizeof(h_cnt), hipMemcpyHostToDevice, s));
  if (m > 0) hipLaunchKernelGGL(k_rmat_diag, dim3((unsigned)((m + 255) / 256)), dim3(256), 0, s, r0, r1, k0);
  hipLaunchKernelGGL(k_rmat_keys, dim3(4096), dim3(256), 0, s, p, r0, r1, k0, d_cnt);
  ok(hipMemcpyAsync(&h_cnt, d_cnt, sizeof(h_cnt), hipMemcpyDeviceToHost, s));
  ok(hipStreamSynchronize(s));
  const int num = (int)h_cnt;
  int end_bit = 32;
  while (end_bit < 64 && ((int64_t)1 << (end_bit - 32)) < m) ++end_bit;
  size_t tb_sort = 0, tb_uniq = 0;
  if (rc == 0) {
    ok(hipcub::DeviceRadixSort::SortKeys(nullptr, tb_sort, k0, k1, num, 0, end_bit, s));
    ok(hipcub::DeviceSelect::Unique(nullptr, tb_uniq, k1, k0, d_nsel, num, s));
  }
  if (rc == 0 && ok(hipMalloc(&tmp, tb_sort > tb_uniq ? tb_sort : tb_uniq))) {
    size_t tb = tb_sort;
    ok(hipcub::DeviceRadixSort::SortKeys(tmp, tb, k0, k1, num, 0, end_bit, s));
    tb = tb_uniq;
    ok(hipcub::DeviceSelect::Unique(tmp, tb, k1, k0, d_nsel, num, s));
  }
  int nsel = 0;
  if (rc == 0) {
    ok(hipMemcpyAsync(&nsel, d_nsel, sizeof(int), hipMemcpyDeviceToHost, s));
    ok(hipStreamSynchronize(s));
  }
  hipFree(tmp);
  hipFree(k1);
  hipFree(d_cnt);
  hipFree(d_nsel);
  if (rc == 0) {
    const int64_t nnz = nsel;
    if (ok(hipMalloc(col_dev, (nnz + kCsrPad) * sizeof(int32_t))) &&
        ok(hipMalloc(val_dev, (nnz + kCsrPad) * sizeof(double)))) {
      ok(hipMemsetAsync(*col_dev + nnz, 0, kCsrPad * sizeof(int32_t), s));
      ok(hipMemsetAsync(*val_dev + nnz, 0, kCsrPad * sizeof(double), s));
      hipLaunchKernelGGL(k_rmat_csr, dim3((unsigned)((nnz + 1 + 255) / 256)), dim3(256), 0, s, k0, nnz,
                         r0, m, p.seed, nplant, plant_dev, p.n, rowptr_dev, *col_dev, *val_dev,
                         p.relabel, p.perm);
      ok(hipGetLastError());
      ok(hipStreamSynchronize(s));
      *nnz_out = nnz;
    }
  }
  hipFree(k0);
  return rc;
}

void col_footprint(const int32_t* col, int64_t nnz, const int64_t* bounds_dev, int P,
                   unsigned long long* lo, unsigned long long* hi, hipStream_t s) {
  if (nnz <= 0) return;
  const int64_t blocks = (nnz + 255) / 256 < 8192 ? (nnz + 255) / 256 : 8192;
  hipLaunchKernelGGL(k_col_footprint, dim3((unsigned)blocks), dim3(256), 0, s, col, nnz, bounds_dev, P, lo, hi);
}

}  // namespace rbl
