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
//   * Everything a tile needs — its CSR col/val segment, its 17 row pointers, the new ring
//     rows, the Q_{i-1} rows of the epilogue and the tile descriptor of the tile two ahead —
//     is fetched by VECTOR loads two tiles ahead into registers and written to a double-
//     buffered LDS stage after the intervening tile computes.  compute() issues no global
//     load, so no vmcnt wait ever drains the prefetch and HBM latency hides behind compute.
//   * one wave per row; its 4 lane groups (16 lanes) each take a contiguous quarter of the
//     row's nonzeros.  A group's lanes read 16 (ring offset, val) pairs with one ds_read
//     each; v_add_u32_dpp / v_fmac_f64_dpp with row_newbcast:s broadcast pair s inside the
//     address add and the FMA themselves (1 VALU + 1 ds_read_b128 + 2 VALU per 4 nonzeros
//     at b = 32).  Each lane owns VEC = b/16 consecutive columns of the row.
//   * group partial sums meet through v_permlane16_swap / v_permlane32_swap; group 0
//     writes the 256-B (b=32) row of U.
// The host (rbl_api.cpp) checks that every tile fits (window_ok); otherwise the general
// gather kernel (spmm.hip) runs.
#include <cstdlib>
#include <type_traits>
#include <utility>

#include <atomic>
#include <mutex>
#include <set>
#include <utility>

#include "kernels.hpp"

namespace rbl {

namespace win {
constexpr int kTileRows = 16;      // rows per tile == waves per workgroup
constexpr int kThreads = 1024;
constexpr int kMeta = 2048;        // (col,val) entries per tile buffer
constexpr int kRingBytes = 65536;  // Q ring
// LDS stage buffer: vals (kMeta*8) | ring offsets (kMeta*4) | Q_{i-1} rows (16*32*8) | rowptr (32*4)
constexpr int kStageVal = 0;
constexpr int kStageOff = kMeta * 8;
constexpr int kStageQp = kStageOff + kMeta * 4;
constexpr int kStageRp = kStageQp + kTileRows * 32 * 8;
constexpr int kStageBytes = kStageRp + 32 * 4;
constexpr size_t kLds = kRingBytes + 2 * (size_t)kStageBytes + 8192;  // + epilogue B_i table
}  // namespace win

template <int S, int N, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (S < N) {
    f(std::integral_constant<int, S>{});
    static_for<S + 1, N>(f);
  }
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
  const int64_t* tinfo;   // per tile: e0, nnz, lo, hi (new ring rows), cmin, cmax, 0, 0
  const double* Q;        // Q row c at Q + (c - col_off) * b
  int64_t col_off;
  double* U;
  const double* Qprev;    // may be null
  const double* Bi;       // b x b row-major (B_i), with Qprev
  int ablate;             // diagnostics only (RBL_SPMM_ABLATE): 1 skip compute, 2 skip data loads
};

// one tile's prefetched data in registers (per thread), plus the descriptor of the tile two
// ahead (lane l holds field l & 7 of it)
struct Stage {
  int c0, c1;
  double v0, v1;
  double q;        // one element of a new ring row
  double qp;       // one element of the tile's Q_{i-1} rows
  int64_t rp;      // rowptr[16 T + tid] (tid <= 16)
  int64_t info_next;  // descriptor field (lane & 7) of the next tile of this stage
  // descriptor of the tile this stage holds, wave-uniform (SGPRs)
  int64_t e0, m, lo, hi, cmin;
};

__device__ __forceinline__ int64_t field(int64_t v, int f) {
  const int lo = __builtin_amdgcn_readlane((int)(v & 0xffffffffll), f);
  const int hi = __builtin_amdgcn_readlane((int)(v >> 32), f);
  return ((int64_t)hi << 32) | (unsigned)lo;
}

template <int VEC, bool EPI>
__global__ __launch_bounds__(win::kThreads) void k_spmm_window(WinArgs a) {
  constexpr int B = 16 * VEC;
  constexpr int RING = win::kRingBytes / (B * 8);
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  double* ring = reinterpret_cast<double*>(smem);
  unsigned char* stage0 = smem + win::kRingBytes;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g = lane >> 4, li = lane & 15;
  const int64_t t0 = (int64_t)blockIdx.x * a.tiles_per_wg;
  const int64_t t1 = t0 + a.tiles_per_wg < a.ntiles ? t0 + a.tiles_per_wg : a.ntiles;
  if (t0 >= t1) return;  // whole workgroup: uniform

  auto ring_off = [](int c) -> int { return (c & (RING - 1)) * (B * 8); };
  auto sval = [&](int buf) { return reinterpret_cast<double*>(stage0 + buf * win::kStageBytes + win::kStageVal); };
  auto soff = [&](int buf) { return reinterpret_cast<int*>(stage0 + buf * win::kStageBytes + win::kStageOff); };
  auto sqp = [&](int buf) { return reinterpret_cast<double*>(stage0 + buf * win::kStageBytes + win::kStageQp); };
  auto srp = [&](int buf) { return reinterpret_cast<int*>(stage0 + buf * win::kStageBytes + win::kStageRp); };

  auto load_info = [&](int64_t t) -> int64_t {
    return t < t1 ? a.tinfo[t * 8 + (lane & 7)] : 0;
  };
  // issue the data loads of tile t (descriptor S.info_next already in registers)
  auto load_stage = [&](int64_t t, Stage& S) {
    S.e0 = field(S.info_next, 0);
    S.m = field(S.info_next, 1);
    S.lo = field(S.info_next, 2);
    S.hi = field(S.info_next, 3);
    S.cmin = field(S.info_next, 4);
    S.info_next = load_info(t + 2);
    S.c0 = S.c1 = 0;
    S.v0 = S.v1 = 0.0;
    S.q = S.qp = 0.0;
    S.rp = 0;
    if (t >= t1) return;
    const int64_t e0 = S.e0, m = S.m, lo = S.lo, hi = S.hi;
    if (a.ablate == 2) {  // diagnostics: row pointers only, metadata / Q rows stay stale
      const int64_t ra = t * win::kTileRows;
      if (tid <= win::kTileRows) S.rp = a.rowptr[ra + tid < a.nrows ? ra + tid : a.nrows];
      return;
    }
    if (tid < m) { S.c0 = a.col[e0 + tid]; S.v0 = a.val[e0 + tid]; }
    if (tid + win::kThreads < m) {
      S.c1 = a.col[e0 + tid + win::kThreads];
      S.v1 = a.val[e0 + tid + win::kThreads];
    }
    const int64_t row = lo + tid / B;
    if (row < hi) S.q = a.Q[(row - a.col_off) * B + (tid % B)];
    const int64_t ra = t * win::kTileRows;
    if (tid <= win::kTileRows) S.rp = a.rowptr[ra + tid < a.nrows ? ra + tid : a.nrows];
    if constexpr (EPI) {
      const int64_t pr = ra + tid / B;
      if (tid < win::kTileRows * B && pr < a.nrows) S.qp = a.Qprev[pr * B + (tid % B)];
    }
  };
  auto store_stage = [&](int64_t t, const Stage& S) {
    if (t >= t1) return;
    const int buf = (int)(t & 1);
    const int64_t e0 = S.e0, m = S.m, lo = S.lo, hi = S.hi;
    // metadata keeps the ring BYTE offset of the column's Q row, not the column id
    if (tid < m) { soff(buf)[tid] = ring_off(S.c0); sval(buf)[tid] = S.v0; }
    if (tid + win::kThreads < m) {
      soff(buf)[tid + win::kThreads] = ring_off(S.c1);
      sval(buf)[tid + win::kThreads] = S.v1;
    }
    const int64_t row = lo + tid / B;
    if (row < hi) ring[(row & (RING - 1)) * B + (tid % B)] = S.q;
    if (tid <= win::kTileRows) srp(buf)[tid] = (int)(S.rp - e0);
    if (tid == 0) srp(buf)[win::kTileRows + 1] = ring_off((int)S.cmin);
    if constexpr (EPI) {
      if (tid < win::kTileRows * B) sqp(buf)[tid] = S.qp;
    }
  };

  // epilogue coefficients: lane owns columns c = li*VEC + v, group g owns t in [g*B/4, (g+1)*B/4)
  // (kept in LDS as a per-lane table [pair][lane] of double2: conflict-free ds_read_b128)
  constexpr int TQ = B / 4;
  constexpr int NBQ = VEC * TQ / 2;  // double2 per lane
  typedef double d2v __attribute__((ext_vector_type(2)));
  d2v* bqs = reinterpret_cast<d2v*>(smem + win::kRingBytes + 2 * win::kStageBytes);
  if constexpr (EPI) {
    if (wave == 0) {
#pragma unroll
      for (int p = 0; p < NBQ; ++p) {
        const int f0 = 2 * p, f1 = 2 * p + 1;
        bqs[p * 64 + lane] = d2v{a.Bi[(li * VEC + f0 / TQ) * B + g * TQ + f0 % TQ],
                                 a.Bi[(li * VEC + f1 / TQ) * B + g * TQ + f1 % TQ]};
      }
    }
  }
  // LDS byte address of this lane's slice of ring row 0 (the dynamic LDS base included)
  typedef __attribute__((address_space(3))) unsigned char lds_u8;
  const unsigned lane_off = (unsigned)(size_t)(lds_u8*)smem + (unsigned)(li * VEC * 8);

  auto compute = [&](int64_t t) {
    if (a.ablate == 1) return;  // diagnostics: pipeline only
    const int64_t r = t * win::kTileRows + wave;
    if (r >= a.nrows) return;  // wave-uniform
    const int buf = (int)(t & 1);
    const int* rp = srp(buf);
    const int* mc = soff(buf);
    const double* mv = sval(buf);
    const int eb = __builtin_amdgcn_readfirstlane(rp[wave]);
    const int m = __builtin_amdgcn_readfirstlane(rp[wave + 1]) - eb;
    const int safe = rp[win::kTileRows + 1];  // a loaded row: masked lanes read finite data
    const int quarter = (m + 3) >> 2;
    const int my_b = eb + g * quarter;
    const int my_e = (g * quarter + quarter < m ? my_b + quarter : eb + m);
    // two accumulator sets (even / odd sub-iteration) shorten the FMA dependency chains
    double acc[2][VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) acc[0][v] = acc[1][v] = 0.0;

    // KB consecutive sub-iterations S0..S0+KB-1: KB address ops and LDS reads issued
    // together, then KB*VEC FMAs; (col, val) broadcasts folded in by DPP row_newbcast
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
        if constexpr (VEC == 2) {
          const d2v d = *(const lds_d2*)(size_t)ad;
          q[decltype(ic)::value][0] = d[0];
          q[decltype(ic)::value][1] = d[1];
        } else {
          q[decltype(ic)::value][0] = *(const lds_d*)(size_t)ad;
        }
      });
      __builtin_amdgcn_sched_barrier(0);  // all KB reads in flight before the FMAs
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
    double sum[VEC];
#pragma unroll
    for (int v = 0; v < VEC; ++v) sum[v] = acc[0][v] + acc[1][v];
    if constexpr (EPI) {
      const double* qp = sqp(buf) + wave * B + g * TQ;
#pragma unroll
      for (int p = 0; p < NBQ; ++p) {
        const d2v bb = bqs[p * 64 + lane];
        const int f0 = 2 * p, f1 = 2 * p + 1;
        sum[f0 / TQ] = fma(-qp[f0 % TQ], bb[0], sum[f0 / TQ]);
        sum[f1 / TQ] = fma(-qp[f1 % TQ], bb[1], sum[f1 / TQ]);
      }
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

  // ---- prologue: tile t0 loads its whole window, then t0 and t0+1 go through the stage ----
  {
    const int64_t lo = field(load_info(t0), 4), hi = field(load_info(t0), 5) + 1;
    for (int64_t e = tid; e < (hi - lo) * B; e += win::kThreads) {
      const int64_t row = lo + e / B;
      ring[(row & (RING - 1)) * B + (e % B)] = a.Q[(row - a.col_off) * B + (e % B)];
    }
    Stage S0;
    S0.info_next = load_info(t0);
    load_stage(t0, S0);
    // t0's new rows were loaded with the full window above: store_stage only rewrites them
    store_stage(t0, S0);
    Stage S1;
    S1.info_next = load_info(t0 + 1);
    load_stage(t0 + 1, S1);
    store_stage(t0 + 1, S1);
  }
  Stage SA, SB;
  SA.info_next = load_info(t0 + 2);
  SB.info_next = load_info(t0 + 3);
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

int window_grid() {
  static std::atomic<int> num_cus[64];  // per device; zero-initialised (static storage)
  int dev = 0;
  (void)hipGetDevice(&dev);
  if (dev < 0 || dev >= 64) dev = 0;
  int n = num_cus[dev].load(std::memory_order_relaxed);
  if (n == 0) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, dev) == hipSuccess) n = p.multiProcessorCount;
    if (n <= 0) n = 256;
    num_cus[dev].store(n, std::memory_order_relaxed);
  }
  return n;
}

void ensure_lds_attr(const void* kernel, int bytes) {
  static std::mutex mu;
  static std::set<std::pair<int, const void*>> done;
  int dev = 0;
  (void)hipGetDevice(&dev);
  std::lock_guard<std::mutex> lk(mu);
  if (done.insert({dev, kernel}).second)
    (void)hipFuncSetAttribute(kernel, hipFuncAttributeMaxDynamicSharedMemorySize, bytes);
}

template <int VEC, bool EPI>
static void launch_window_t(const WinArgs& a, int grid, hipStream_t s) {
  ensure_lds_attr(reinterpret_cast<const void*>(&k_spmm_window<VEC, EPI>), (int)win::kLds);
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
  a.tinfo = A.tile_info;
  a.Q = Qin;
  a.col_off = col_off;
  a.U = U;
  a.Qprev = Qprev;
  a.Bi = Bi;
#ifdef RBL_VARIANTS
  static const int ablate = [] {  // diagnostics: 1 skip compute, 2 skip data loads
    const char* e = getenv("RBL_SPMM_ABLATE");
    return e ? atoi(e) : 0;
  }();
  a.ablate = ablate;
#else
  a.ablate = 0;
#endif
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
