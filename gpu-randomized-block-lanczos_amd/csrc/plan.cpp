// plan.cpp — host-only planning entry points of librbl_hip.so (no GPU needed).
//
// The reference has no partitioning (single GPU); its memory planning is
// gpu_buffer_size / blocksize (Julia/RBL_gpu.jl:24-27, 95-104), which the HIP path replaces by
// keeping the whole basis in HBM.  These functions size the row-partitioned multi-GPU job.
#include <algorithm>
#include <cstdint>
#include <vector>

#include "../../include/rbl_hip.h"
#include "rbl_common.hpp"

extern "C" {

int rbl_plan_row_partition(int64_t n, const int64_t* rowptr, int nranks, int64_t* bounds_out) {
  if (n < 0 || nranks < 1 || !rowptr || !bounds_out) return RBL_ERR_INVALID;
  // balance nnz + rows (rows carry the tall-skinny work, nnz the SpMM work)
  const int64_t nnz = rowptr[n] - rowptr[0];
  const double total = (double)nnz + (double)n;
  bounds_out[0] = 0;
  int64_t r = 0;
  for (int p = 1; p < nranks; ++p) {
    const double target = total * p / nranks;
    while (r < n && (double)(rowptr[r] - rowptr[0]) + (double)r < target) ++r;
    bounds_out[p] = std::max(r, bounds_out[p - 1]);
  }
  bounds_out[nranks] = n;
  return RBL_OK;
}

int rbl_plan_halo(int64_t nrows_local, const int64_t* rowptr, const int64_t* colind,
                  int index_base, int nranks, const int64_t* bounds, int64_t* lo, int64_t* hi) {
  if (nrows_local < 0 || !rowptr || nranks < 1 || !bounds || !lo || !hi) return RBL_ERR_INVALID;
  const int64_t nnz = rowptr[nrows_local] - rowptr[0];
  if (nnz > 0 && !colind) return RBL_ERR_INVALID;
  std::vector<int64_t> mn(nranks, INT64_MAX), mx(nranks, -1);
  const int64_t e0 = rowptr[0] - index_base;
  for (int64_t e = 0; e < nnz; ++e) {
    const int64_t c = colind[e0 + e] - index_base;
    const int q = (int)(std::upper_bound(bounds, bounds + nranks + 1, c) - bounds) - 1;
    if (q < 0 || q >= nranks) return RBL_ERR_INVALID;
    mn[q] = std::min(mn[q], c);
    mx[q] = std::max(mx[q], c + 1);
  }
  for (int q = 0; q < nranks; ++q) {
    lo[q] = mx[q] < 0 ? 0 : mn[q];
    hi[q] = mx[q] < 0 ? 0 : mx[q];
  }
  return RBL_OK;
}

int rbl_hashwindow_rows_host(int64_t n, int64_t halfwidth, double density, uint64_t seed,
                             int nplant, const double* plant, int64_t row_begin, int64_t row_end,
                             int64_t* rowptr_out, int64_t* colind_out, double* val_out) {
  if (n < 1 || halfwidth < 0 || row_begin < 0 || row_end > n || row_end < row_begin ||
      !rowptr_out || nplant < 0 || (nplant > 0 && !plant))
    return RBL_ERR_INVALID;
  const int64_t stride = nplant > 0 ? n / nplant : 0;
  int64_t e = 0;
  rowptr_out[0] = 0;
  for (int64_t r = row_begin; r < row_end; ++r) {
    const int64_t lo = std::max<int64_t>(0, r - halfwidth);
    const int64_t hi = std::min<int64_t>(n - 1, r + halfwidth);
    for (int64_t c = lo; c <= hi; ++c) {
      double v;
      if (c == r) {
        v = rbl::hw_value(seed, r, r);
        if (stride > 0 && r % stride == 0 && r / stride < nplant) v += plant[r / stride];
      } else {
        const int64_t a = std::min(r, c), b = std::max(r, c);
        if (!rbl::hw_present(seed, a, b, density)) continue;
        v = rbl::hw_value(seed, a, b);
      }
      if (colind_out) colind_out[e] = c;
      if (val_out) val_out[e] = v;
      ++e;
    }
    rowptr_out[r - row_begin + 1] = e;
  }
  return RBL_OK;
}

}  // extern "C"
