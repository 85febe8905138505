// spmm_window.hip — persistent LDS-window CSR SpMM for banded / windowed sparsity (gfx950).
//
// U = A * Q_i  (+ fused 3-term epilogue U -= Q_{i-1} B_i^T), replacing cuSPARSE SpMM and the
// following cuBLAS gemm of RBL_gpu.jl:176-177.  HBM-bound: algorithmic bytes per call
// nnz*(8+4) + (n+1)*8 + 2*n*b*8 (+ n*b*8 for Q_{i-1}).
//
// Structure (one 1024-thread workgroup per CU, persistent over a contiguous range of
// 16-row tiles):
//   * LDS ring of Q rows (64 KB): slot = global row & (RING-1); each tile only loads the
//     rows its window adds, so Q is read ~once from HBM (plus one halo per CU).
//   * tile metadata (the CSR col/val segment of 16 rows) double-buffered in LDS, staged
//     through registers two tiles ahead (prefetch distance 2 tiles) so HBM latency hides
//     behind the compute of the intervening tiles.
//   * one wave per row; its 4 lane groups (16 lanes) each take a contiguous quarter of
//     the row's nonzeros.  A group's 16 lanes read 16 (col,val) pairs from LDS with one
//     ds_read each, then DPP row_newbcast:s broadcasts pair s to the group — the per-
//     nonzero metadata costs 3 VALU movs and no LDS bandwidth.  Each lane owns VEC = b/16
//     consecutive columns: one ds_read_b128 (b=32) / ds_read_b64 (b=16) of the Q row per
//     nonzero, VEC fp64 FMAs.
//   * group partial sums meet through v_permlane16_swap / v_permlane32_swap; group 0
//     writes the 256-B (b=32) row of U.
// The host (rbl_api.cpp) validates that every tile fits (window_ok); otherwise the
// general gather kernel (spmm.hip) runs.
#include <type_traits>
#include <utility>

#include "kernels.hpp"

namespace rbl {

namespace win {
constexpr int kTileRows = 16;      // rows per tile == waves per workgroup
constexpr int kThreads = 1024;
constexpr int kMeta = 2048;        // (col,val) entries per tile buffer
constexpr int kRingBytes = 65536;  // Q ring
constexpr size_t kLds = kRingBytes + 2 * (size_t)kMeta * (8 + 4);
}  // namespace win

template <int S, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (S < N) {
    f(std::integral_constant<int, S>{});
    static_for<S + 1, N>(f);
  }
}

template <int S>
__device__ __forceinline__ int bcast_i(int x) {
  return __builtin_amdgcn_mov_dpp(x, 0x150 + S, 0xF, 0xF, false);  // row_newbcast:S
}
template <int S>
__device__ __forceinline__ double bcast_d(double x) {
  const long long u = __builtin_bit_cast(long long, x);
  const int lo = bcast_i<S>((int)(u & 0xffffffffll));
  const int hi = bcast_i<S>((int)(u >> 32));
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned int)lo);
}
// dpp(off) + lane_off with off taken from lane S of the lane's 16-lane row
template <int S>
__device__ __forceinline__ unsigned add_bcast(unsigned off, unsigned lane_off) {
  unsigned r;
  asm("v_add_u32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
      : "=v"(r)
      : "v"(off), "v"(lane_off), "n"(S));
  return r;
}
// acc += dpp(val) * q with val taken from lane S of the lane's 16-lane row
template <int S>
__device__ __forceinline__ void fmac_bcast(double& acc, double val, double q) {
  asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
      : "+v"(acc)
      : "v"(val), "v"(q), "n"(S));
}

// sum over the 4 lane groups (16-lane rows) of the wave; every lane gets the total
__device__ __forceinline__ double group_sum(double x) {
  long long u = __builtin_bit_cast(long long, x);
  unsigned lo = (unsigned)(u & 0xffffffffll), hi = (unsigned)(u >> 32);
  auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  double a = __builtin_bit_cast(double, ((unsigned long long)h16[0] << 32) | l16[0]);
  double b = __builtin_bit_cast(double, ((unsigned long long)h16[1] << 32) | l16[1]);
  double s = a + b;
  u = __builtin_bit_cast(long long, s);
  lo = (unsigned)(u & 0xffffffffll);
  hi = (unsigned)(u >> 32);
  auto l32 = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
  auto h32 = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
  a = __builtin_bit_cast(double, ((unsigned long long)h32[0] << 32) | l32[0]);
  b = __builtin_bit_cast(double, ((unsigned long long)h32[1] << 32) | l32[1]);
  return a + b;
}

struct WinArgs {
  int64_t nrows;
  int64_t ntiles;
  int64_t tiles_per_wg;
  const int64_t* rowptr;
  const int32_t* col;
  const double* val;
  const int64_t* tcmin;   // per tile, forward-filled, non-decreasing
  const int64_t* tcmax;
  const double* Q;        // Q row c at Q + (c - col_off) * b
  int64_t col_off;
  double* U;
  const double* Qprev;    // may be null
  const double* Bi;       // b x b row-major (B_i), with Qprev
};

// registers holding one tile's prefetched data (per thread)
struct Stage {
  int c0, c1;
  double v0, v1;
  double q;
};

template <int VEC, bool EPI>
__global__ __launch_bounds__(win::kThreads) void k_spmm_window(WinArgs a) {
  constexpr int B = 16 * VEC;
  constexpr int RING = win::kRingBytes / (B * 8);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* ring = reinterpret_cast<double*>(smem);
  double* mval0 = reinterpret_cast<double*>(smem + win::kRingBytes);
  int32_t* mcol0 = reinterpret_cast<int32_t*>(smem + win::kRingBytes + 2 * win::kMeta * 8);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int64_t t0 = (int64_t)blockIdx.x * a.tiles_per_wg;
  const int64_t t1 = t0 + a.tiles_per_wg < a.ntiles ? t0 + a.tiles_per_wg : a.ntiles;
  if (t0 >= t1) return;  // whole workgroup: uniform

  auto tile_e = [&](int64_t t, int64_t& e0, int64_t& e1) {
    const int64_t ra = t * win::kTileRows;
    const int64_t rb = ra + win::kTileRows < a.nrows ? ra + win::kTileRows : a.nrows;
    e0 = a.rowptr[ra];
    e1 = a.rowptr[rb];
  };
  // new ring rows of tile t: [lo, hi)
  auto tile_new = [&](int64_t t, int64_t& lo, int64_t& hi) {
    hi = a.tcmax[t] + 1;
    lo = a.tcmin[t];
    if (t > t0) {
      const int64_t ph = a.tcmax[t - 1] + 1;
      lo = lo > ph ? lo : ph;
    }
  };
  auto ring_off = [](int c) -> int { return (c & (RING - 1)) * (B * 8); };
  auto load_stage = [&](int64_t t, Stage& S) {
    S.c0 = S.c1 = 0;
    S.v0 = S.v1 = 0.0;
    S.q = 0.0;
    if (t >= t1) return;
    int64_t e0, e1, lo, hi;
    tile_e(t, e0, e1);
    const int64_t i0 = e0 + tid, i1 = e0 + tid + win::kThreads;
    if (i0 < e1) { S.c0 = a.col[i0]; S.v0 = a.val[i0]; }
    if (i1 < e1) { S.c1 = a.col[i1]; S.v1 = a.val[i1]; }
    tile_new(t, lo, hi);
    const int64_t row = lo + tid / B;
    if (row < hi) S.q = a.Q[(row - a.col_off) * B + (tid % B)];
  };
  auto store_stage = [&](int64_t t, const Stage& S) {
    if (t >= t1) return;
    int64_t e0, e1, lo, hi;
    tile_e(t, e0, e1);
    const int buf = (int)(t & 1);
    int32_t* mc = mcol0 + buf * win::kMeta;
    double* mv = mval0 + buf * win::kMeta;
    const int64_t m = e1 - e0;
    // metadata keeps the ring BYTE offset of the column's Q row, not the column id
    if (tid < m) { mc[tid] = ring_off(S.c0); mv[tid] = S.v0; }
    if (tid + win::kThreads < m) {
      mc[tid + win::kThreads] = ring_off(S.c1);
      mv[tid + win::kThreads] = S.v1;
    }
    tile_new(t, lo, hi);
    const int64_t row = lo + tid / B;
    if (row < hi) ring[(row & (RING - 1)) * B + (tid % B)] = S.q;
  };

  // epilogue coefficients: lane owns columns c = li*VEC + v, group g owns t in [g*B/4, (g+1)*B/4)
  constexpr int TQ = B / 4;
  double bq[EPI ? VEC : 1][EPI ? TQ : 1];
  if constexpr (EPI) {
#pragma unroll
    for (int v = 0; v < VEC; ++v)
#pragma unroll
      for (int j = 0; j < TQ; ++j) bq[v][j] = a.Bi[(li * VEC + v) * B + g * TQ + j];
  }

  auto compute = [&](int64_t t) {
    const int64_t r = t * win::kTileRows + wave;
    if (r >= a.nrows) return;  // wave-uniform
    const int buf = (int)(t & 1);
    const int32_t* mc = mcol0 + buf * win::kMeta;
    const double* mv = mval0 + buf * win::kMeta;
    const int64_t tb = a.rowptr[t * win::kTileRows];
    const int64_t rs = a.rowptr[r], re = a.rowptr[r + 1];
    const int m = (int)(re - rs);
    const int eb = (int)(rs - tb);
    const int quarter = (m + 3) >> 2;
    const int my_b = eb + g * quarter;
    const int my_e = (g * quarter + quarter < m ? my_b + quarter : eb + m);
    const int safe = ring_off((int)a.tcmin[t]);  // a loaded row: masked lanes read finite data
    // LDS byte address of this lane's slice of ring row 0 (the dynamic LDS base included)
    typedef __attribute__((address_space(3))) unsigned char lds_u8;
    const unsigned lds_base = (unsigned)(size_t)(lds_u8*)smem;
    const unsigned lane_off = lds_base + (unsigned)(li * VEC * 8);
    // two accumulator sets (even / odd sub-iteration) shorten the FMA dependency chains
    double acc[2][VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[0][v] = acc[1][v] = 0.0;

    // KB consecutive sub-iterations S0..S0+KB-1: KB address ops, KB LDS reads, KB*VEC FMAs,
    // every (col, val) broadcast folded into the instruction by DPP row_newbcast
    auto block = [&](int cl, double vl, auto s0, auto kb) {
      constexpr int S0 = decltype(s0)::value;
      constexpr int KB = decltype(kb)::value;
      double q[KB][VEC];
      static_for<0, KB>([&](auto ic) {
        constexpr int S = S0 + decltype(ic)::value;
        const unsigned ad = add_bcast<S>((unsigned)cl, lane_off);
        typedef __attribute__((address_space(3))) const double lds_d;
        typedef double d2v __attribute__((ext_vector_type(2)));
        typedef __attribute__((address_space(3))) const d2v lds_d2;
        const lds_d* qp = (const lds_d*)(size_t)ad;
        if constexpr (VEC == 2) {
          const d2v d = *(const lds_d2*)(size_t)ad;
          q[decltype(ic)::value][0] = d[0];
          q[decltype(ic)::value][1] = d[1];
        } else {
          q[decltype(ic)::value][0] = qp[0];
        }
      });
      static_for<0, KB>([&](auto ic) {
        constexpr int S = S0 + decltype(ic)::value;
#pragma unroll
        for (int v = 0; v < VEC; ++v) fmac_bcast<S>(acc[S & 1][v], vl, q[decltype(ic)::value][v]);
      });
    };
    for (int c0 = 0; c0 < quarter; c0 += 16) {
      const int idx = my_b + c0 + li;
      const bool ok = idx < my_e;
      int cl = ok ? mc[idx] : safe;
      double vl = ok ? mv[idx] : 0.0;
      // VALU write -> DPP read needs 2 wait states; hipcc does not pad inside asm
      asm volatile("s_nop 1" : "+v"(cl), "+v"(vl));
      const int nsub = quarter - c0;
      if (nsub >= 16) {
        block(cl, vl, std::integral_constant<int, 0>{}, std::integral_constant<int, 8>{});
        block(cl, vl, std::integral_constant<int, 8>{}, std::integral_constant<int, 8>{});
      } else {
        // tail: blocks of 4 (masked lanes contribute 0 * finite)
        static_for<0, 4>([&](auto h) {
          constexpr int H = decltype(h)::value;
          if (H * 4 < nsub)
            block(cl, vl, std::integral_constant<int, H * 4>{}, std::integral_constant<int, 4>{});
        });
      }
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[0][v] += acc[1][v];
    double* sum = acc[0];
    if constexpr (EPI) {
      const double* qp = a.Qprev + r * B + g * TQ;
      double qv[TQ];
#pragma unroll
      for (int j = 0; j < TQ; ++j) qv[j] = qp[j];
#pragma unroll
      for (int v = 0; v < VEC; ++v)
#pragma unroll
        for (int j = 0; j < TQ; ++j) sum[v] = fma(-qv[j], bq[v][j], sum[v]);
    }
#pragma unroll
    for (int v = 0; v < VEC; ++v) sum[v] = group_sum(sum[v]);
    if (g == 0) {
      double* up = a.U + r * B + li * VEC;
      if constexpr (VEC == 2) {
        *reinterpret_cast<double2*>(up) = double2{sum[0], sum[1]};
      } else {
        up[0] = sum[0];
      }
    }
  };

  // ---- prologue: tile t0 (full window) and t0+1 go straight to LDS ----
  {
    const int64_t lo = a.tcmin[t0], hi = a.tcmax[t0] + 1;
    for (int64_t e = tid; e < (hi - lo) * B; e += win::kThreads) {
      const int64_t row = lo + e / B;
      ring[(row & (RING - 1)) * B + (e % B)] = a.Q[(row - a.col_off) * B + (e % B)];
    }
    int64_t e0, e1;
    tile_e(t0, e0, e1);
    const int buf0 = (int)(t0 & 1);  // compute(t) reads buffer t & 1
    for (int64_t e = tid; e < e1 - e0; e += win::kThreads) {
      mcol0[buf0 * win::kMeta + e] = ring_off(a.col[e0 + e]);
      mval0[buf0 * win::kMeta + e] = a.val[e0 + e];
    }
    Stage S1;
    load_stage(t0 + 1, S1);
    store_stage(t0 + 1, S1);
  }
  Stage SA, SB;
  load_stage(t0 + 2, SA);
  load_stage(t0 + 3, SB);
  __syncthreads();

  // ---- steady state: prefetch distance two tiles ----
  for (int64_t t = t0; t < t1; t += 2) {
    compute(t);
    __syncthreads();
    store_stage(t + 2, SA);
    load_stage(t + 4, SA);
    if (t + 1 < t1) {
      compute(t + 1);
      __syncthreads();
      store_stage(t + 3, SB);
      load_stage(t + 5, SB);
    }
  }
}

static int g_num_cus = 0;

int window_grid() {
  if (g_num_cus == 0) {
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess) g_num_cus = p.multiProcessorCount;
    if (g_num_cus <= 0) g_num_cus = 256;
  }
  return g_num_cus;
}

template <int VEC, bool EPI>
static void launch_window_t(const WinArgs& a, int grid, hipStream_t s) {
  static bool attr = false;
  if (!attr) {
    hipFuncSetAttribute(reinterpret_cast<const void*>(&k_spmm_window<VEC, EPI>),
                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)win::kLds);
    attr = true;
  }
  hipLaunchKernelGGL((k_spmm_window<VEC, EPI>), dim3(grid), dim3(win::kThreads), win::kLds, s, a);
}

bool spmm_window(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
                 const double* Qprev, const double* Bi, hipStream_t s) {
  if (A.ntiles <= 0 || !((b == 16 && A.window_ok16) || (b == 32 && A.window_ok32))) return false;
  WinArgs a;
  a.nrows = A.nrows;
  a.ntiles = A.ntiles;
  a.tiles_per_wg = A.tiles_per_wg;
  a.rowptr = A.rowptr;
  a.col = A.col;
  a.val = A.val;
  a.tcmin = A.tile_cmin;
  a.tcmax = A.tile_cmax;
  a.Q = Qin;
  a.col_off = col_off;
  a.U = U;
  a.Qprev = Qprev;
  a.Bi = Bi;
  const int grid = (int)((A.ntiles + A.tiles_per_wg - 1) / A.tiles_per_wg);
  const bool epi = Qprev != nullptr;
  if (b == 32) {
    if (epi) launch_window_t<2, true>(a, grid, s); else launch_window_t<2, false>(a, grid, s);
  } else {
    if (epi) launch_window_t<1, true>(a, grid, s); else launch_window_t<1, false>(a, grid, s);
  }
  return true;
}

}  // namespace rbl
