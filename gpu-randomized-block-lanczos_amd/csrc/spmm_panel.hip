// spmm_panel.hip — column-panel CSR SpMM for wide bands (gfx950), b = 32, fp64.
//
// U = A * Q_i  (+ the 3-term epilogue U -= Q_{i-1} B_i^T), RBL_gpu.jl:176-177, for matrices
// whose rows reach further than the band-tile (|c - r| <= 64) and LDS-window (a 256-row ring)
// kernels allow — the FEM / circuit orderings of the reference's benchmark.jl:21-28 inputs,
// bandwidths in the hundreds to thousands.  HBM-bound on the CSR stream: per launch
// nnz * (8 + 4) + (n + 1) * 8 + n * b * 8 * (2 + EPI) bytes.
//
// A workgroup (1024 threads, one per CU, persistent) owns row blocks of kRows = 256 rows.  A
// block's columns span [cmin, cmax]; that window is walked in column panels of kPanel = 256 Q
// rows (64 KiB at b = 32), double-buffered in LDS: while panel p is multiplied, panel p + 1 (or
// the next block's first panel) is loaded into registers, written to the other buffer after,
// and one barrier per panel swaps them.  Every Q row a block needs is read from L2 / HBM once
// per block and then from LDS once per nonzero (the 256 B of a Q row per nonzero are the
// kernel's main traffic: ds_read_b128, 256 B/clk/CU).
//
//   * rows: 16-lane group G = tid / 16 (64 per workgroup) owns rows G, G + 64, G + 128, G + 192
//     of the block; lane li holds columns 2 li, 2 li + 1 of each row's accumulator (16 VGPRs)
//   * a row's nonzeros are column-sorted, so its entries in panel p are a prefix of what is
//     left: the group holds a chunk of the next 32 entries (lane li: entries li, 16 + li), a
//     ballot against the panel's end gives the count, the cursor advances by it, and the
//     chunk for the next panel is loaded right after (unconditionally: the row end is applied
//     where the chunk is used) — one panel of latency cover
//   * per entry: v_add_u32_dpp forms the Q row's LDS address from the broadcast offset
//     (row_newbcast), one ds_read_b128, and two v_fmac_f64_dpp with the broadcast value; the
//     four groups of a wave step through their rows' counts together (the wave loops to the
//     largest, masked entries multiply a zero row of finite data)
//   * the epilogue (B_i^T as a per-lane LDS table) and the store of U end a block.
// Work goes to the workgroups XCD by XCD: the 8 XCDs take contiguous eighths of the blocks and
// an XCD's 32 workgroups sweep theirs side by side, so neighbouring blocks — whose windows
// overlap by 2H rows — read their shared panels from the same L2.
#include <cstdint>
#include <type_traits>
#include <utility>

#include "kernels.hpp"

namespace rbl {

namespace pnl {
constexpr int kThreads = 1024;
constexpr int kRows = 256;                       // rows per block
constexpr int kPanel = 256;                      // Q rows per panel
constexpr int kB = 32;
constexpr int kRowBytes = kB * 8;                // 256
constexpr int kPanelBytes = kPanel * kRowBytes;  // 64 KiB
constexpr int kBtBytes = kB * 16 * 16;           // B_i^T table: [u][lane] double2
constexpr size_t kLds = 2 * (size_t)kPanelBytes + kBtBytes;
constexpr int kXcds = 8;
}  // namespace pnl

namespace {

template <int S, int N, class F>
__device__ __forceinline__ void pfor(F&& f) {
  if constexpr (S < N) {
    f(std::integral_constant<int, S>{});
    pfor<S + 1, N>(f);
  }
}
// off (from lane S of the lane's 16-lane row) + lane_off
template <int S>
__device__ __forceinline__ unsigned pnl_addr(unsigned off, unsigned lane_off) {
  unsigned r;
  asm("v_add_u32_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
      : "=v"(r)
      : "v"(off), "v"(lane_off), "n"(S));
  return r;
}
// acc += val (from lane S of the lane's 16-lane row) * q
template <int S>
__device__ __forceinline__ void pnl_fma(double& acc, double val, double q) {
  asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf"
      : "+v"(acc)
      : "v"(val), "v"(q), "n"(S));
}

}  // namespace

struct PanelArgs {
  int64_t nrows;             // local rows
  int64_t nblk;              // blocks of kRows rows
  const int64_t* rowptr;
  const int32_t* col;
  const double* val;
  const int32_t* bpan;       // per block: first and last panel (global panel ids)
  const double* Q;           // Q row c at Q + (c - col_off) * 32, rows [q_lo, q_hi)
  int64_t col_off, q_lo, q_hi;
  const double* zrow;        // >= 32 zeros: the panel rows outside [q_lo, q_hi)
  double* U;
  const double* Qprev;       // may be null (no epilogue)
  const double* Bi;          // b x b row-major (B_i), with Qprev
};

template <bool EPI>
__global__ __launch_bounds__(pnl::kThreads) void k_spmm_panel(PanelArgs a) {
  using namespace pnl;
  typedef double d2v __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) const d2v lds_d2;
  typedef __attribute__((address_space(3))) unsigned char lds_u8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int li = lane & 15;
  const int grp = tid >> 4;                  // 0..63
  const int gw = lane >> 4;                  // group within the wave

  // ---- this workgroup's blocks: XCD x (= blockIdx % 8) takes blocks [x nblk / 8, (x+1) nblk / 8)
  // and its workgroups j = blockIdx / 8 take every (gridDim / 8)-th of them ----
  const int nper = gridDim.x / kXcds;
  const int xcd = blockIdx.x % kXcds, j = blockIdx.x / kXcds;
  const int64_t xb0 = a.nblk * xcd / kXcds, xb1 = a.nblk * (xcd + 1) / kXcds;
  int64_t blk = xb0 + j;
  if (blk >= xb1) return;  // whole workgroup: uniform

  // ---- LDS: the B_i^T table (the panel buffers are written whole, out-of-range rows as
  // zeros, before any read: masked entries read finite data) ----
  {
    if constexpr (EPI) {
      d2v* bt = reinterpret_cast<d2v*>(smem + 2 * kPanelBytes);
      for (int e = tid; e < kB * 16; e += kThreads) {
        const int u = e >> 4, l = e & 15;
        bt[e] = d2v{a.Bi[(2 * l) * kB + u], a.Bi[(2 * l + 1) * kB + u]};
      }
    }
  }
  const unsigned lds_base = (unsigned)(size_t)(lds_u8*)smem;
  const unsigned lane_off = (unsigned)(li * 16);

  // ---- panel staging: LDS-DMA (global_load_lds_dwordx4), no staging registers.  Wave w's
  // instruction i writes 1 KiB = rows 4 (w + 16 i) .. + 3 of the panel (lane l: row + l / 16,
  // bytes 16 (l % 16)); rows outside [q_lo, q_hi) come from a zero row ----
  const int wave = tid >> 6;
  auto load_panel = [&](int p, int buf) {
    const int64_t cb = (int64_t)p * kPanel;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = 4 * (wave + 16 * i);
      const int64_t c = cb + rl + (lane >> 4);
      const double* src = (c >= a.q_lo && c < a.q_hi) ? a.Q + (c - a.col_off) * kB + 2 * li
                                                      : a.zrow + 2 * li;
      __builtin_amdgcn_global_load_lds(src, smem + buf * kPanelBytes + rl * kRowBytes, 16, 0, 0);
    }
  };

  // per row k of the group: cursor and end (relative to the block's first nonzero, nzb), the
  // chunk (entries cur + li, cur + 16 + li), the accumulators
  int cur[4], end[4];
  int c0[4], c1[4];
  double v0[4], v1[4];
  double acc[4][2];
  int ncur[4], nend[4];  // the next block's rows (loaded during the current block)
  auto row_of = [&](int64_t b, int k) -> int64_t { return b * kRows + grp + 64 * k; };
  // block-uniform values through the scalar cache (read-only here): a block's first nonzero
  // and its panel range — s_load, so waiting for them never drains the vector loads in flight
  typedef __attribute__((address_space(4))) const int64_t c_i64;
  typedef __attribute__((address_space(4))) const int32_t c_i32;
  c_i64* rp_s = (c_i64*)a.rowptr;
  c_i32* bp_s = (c_i32*)a.bpan;
  auto block_base = [&](int64_t b) -> int64_t {
    const int64_t r = b * kRows;
    return rp_s[r < a.nrows ? r : a.nrows];
  };
  // a block's row bounds, low 32 bits of rowptr (the differences to the block's first
  // nonzero fit: a block holds < 2^31 nonzeros), made relative to the base where they are used
  const int* rp32 = reinterpret_cast<const int*>(a.rowptr);
  auto load_bounds = [&](int64_t b, int (&cu)[4], int (&en)[4]) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // (rows past the slice: an empty range)
      const int64_t r = row_of(b, k);
      const bool in = r < a.nrows;
      cu[k] = rp32[2 * (in ? r : a.nrows)];
      en[k] = rp32[2 * (in ? r + 1 : a.nrows)];
    }
  };
  int64_t nzb = block_base(blk), nzb_next = 0;
  // unconditional loads (no branches, no early use: the row end is applied in phase A): past
  // a row's end they read the next rows' entries or the CSR's kCsrPad padding, never past it
  // Non-temporal: the CSR streams through once, so its lines leave L2 first and the Q panels
  // — each read by the ~(2H + 256) / 256 workgroups whose windows hold it, a panel step apart —
  // stay there for them.
  auto load_chunk = [&](int k, int64_t base) {
    const int64_t e = base + cur[k] + li;
    c0[k] = __builtin_nontemporal_load(a.col + e);
    v0[k] = __builtin_nontemporal_load(a.val + e);
    c1[k] = __builtin_nontemporal_load(a.col + e + 16);
    v1[k] = __builtin_nontemporal_load(a.val + e + 16);
  };

  int p0 = bp_s[2 * blk], p1 = bp_s[2 * blk + 1];
  int p = p0;
  int buf = 0;
  load_bounds(blk, cur, end);
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    cur[k] -= (int)nzb;
    end[k] -= (int)nzb;
    load_chunk(k, nzb);
    acc[k][0] = acc[k][1] = 0.0;
  }
  load_panel(p, 0);
  __syncthreads();  // (waits for the DMA: an LDS-DMA is a pending load)

  for (;;) {
    // ---- the next step: panel p + 1 of this block, or the next block's first panel ----
    const bool last_panel = p == p1;
    const int64_t nblk = blk + nper;
    const bool have_next = !last_panel || nblk < xb1;
    int np0 = 0, np1 = 0;
    if (last_panel && nblk < xb1) {
      np0 = bp_s[2 * nblk];
      np1 = bp_s[2 * nblk + 1];
    }
    const int pn = last_panel ? np0 : p + 1;
    const int64_t pbase = (int64_t)p * kPanel, pend = pbase + kPanel;
    const unsigned bufb = lds_base + (unsigned)(buf * kPanelBytes);

    // ---- phase A: every row's chunk against the panel's end — counts, LDS offsets, masked
    // values — before the next panel's DMA is issued (hipcc drains an in-flight LDS-DMA at the
    // first use of an ordinary load's result, so the chunks are consumed first) ----
    int m[4], mmax[4];
    unsigned o0[4], o1[4];
    double w0[4], w1[4];
    bool ok0[4], ok1[4];
    auto count = [&](int k) {
      const uint64_t b0 = __ballot(ok0[k]), b1 = __ballot(ok1[k]);
      const int sh = 16 * gw;
      m[k] = __popcll((b0 >> sh) & 0xffffull) + __popcll((b1 >> sh) & 0xffffull);
      int mx = 0;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const int mg = __popcll((b0 >> (16 * g)) & 0xffffull) + __popcll((b1 >> (16 * g)) & 0xffffull);
        mx = mg > mx ? mg : mx;
      }
      mmax[k] = mx;
      // LDS byte offsets of the entries' Q rows in this panel; masked: row 0, value 0
      o0[k] = ok0[k] ? bufb + (unsigned)((c0[k] - pbase) * kRowBytes) : bufb;
      o1[k] = ok1[k] ? bufb + (unsigned)((c1[k] - pbase) * kRowBytes) : bufb;
      w0[k] = ok0[k] ? v0[k] : 0.0;
      w1[k] = ok1[k] ? v1[k] : 0.0;
    };
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ok0[k] = cur[k] + li < end[k] && c0[k] < pend;
      ok1[k] = cur[k] + 16 + li < end[k] && c1[k] < pend;
      count(k);
    }
    __builtin_amdgcn_sched_barrier(0);
    if (have_next) load_panel(pn, buf ^ 1);
    asm volatile("" ::: "memory");  // the loads below stay younger than the DMA
    if (p == p0 && nblk < xb1) {
      nzb_next = block_base(nblk);
      load_bounds(nblk, ncur, nend);
    }

    // ---- phase B: multiply panel p (buffer buf), row by row; each row's chunk for the next
    // step is loaded as soon as its entries here are done ----
    pfor<0, 4>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      for (;;) {
        unsigned u0 = o0[k], u1 = o1[k];
        double x0 = w0[k], x1 = w1[k];
        // VALU write -> DPP read needs 2 wait states; hipcc does not pad inside asm
        asm volatile("s_nop 1" : "+v"(u0), "+v"(u1), "+v"(x0), "+v"(x1));
        double& a0 = acc[k][0];
        double& a1 = acc[k][1];
        const int mx = mmax[k];
        // entries 4h .. 4h + 3 of one chunk register (lanes 4h .. 4h + 3 of the group): their
        // four LDS reads issued together, then their FMAs
        auto quad = [&](unsigned off, double w, auto hh) {
          constexpr int H = decltype(hh)::value;
          d2v q[4];
          pfor<0, 4>([&](auto ic) {
            constexpr int S = 4 * H + decltype(ic)::value;
            q[decltype(ic)::value] = *(lds_d2*)(size_t)pnl_addr<S>(off, lane_off);
          });
          __builtin_amdgcn_sched_barrier(0);  // all four reads in flight before the FMAs
          pfor<0, 4>([&](auto ic) {
            constexpr int S = 4 * H + decltype(ic)::value;
            pnl_fma<S>(a0, w, q[decltype(ic)::value][0]);
            pnl_fma<S>(a1, w, q[decltype(ic)::value][1]);
          });
        };
        pfor<0, 4>([&](auto hh) {
          if (4 * decltype(hh)::value < mx) quad(u0, x0, hh);
        });
        pfor<0, 4>([&](auto hh) {
          if (16 + 4 * decltype(hh)::value < mx) quad(u1, x1, hh);
        });
        cur[k] += m[k];
        // a full chunk may leave entries in this panel: that group loads the next 32 (rare at
        // ~100 nonzeros per row over several panels)
        const bool need = m[k] == 32 && cur[k] < end[k];
        if (__ballot(need) == 0) break;
        if (need) load_chunk(k, nzb);
        ok0[k] = need && cur[k] + li < end[k] && c0[k] < pend;
        ok1[k] = need && cur[k] + 16 + li < end[k] && c1[k] < pend;
        count(k);
      }
      // the row's entries for the next step: the next panel's (the rest of this chunk comes
      // back from L1 / L2), or at a block's last panel the next block's row k
      if (last_panel && nblk < xb1) {
        cur[k] = ncur[k] - (int)nzb_next;
        end[k] = nend[k] - (int)nzb_next;
        load_chunk(k, nzb_next);
      } else if (have_next) {
        load_chunk(k, nzb);
      }
    });
    if (last_panel && nblk < xb1) nzb = nzb_next;

    // ---- block end: epilogue, store U, the next block's accumulators ----
    if (last_panel) {
      // the epilogue's Q_{i-1} rows, one row ahead
      auto qprev_row = [&](int k) -> d2v {
        const int64_t r = row_of(blk, k);
        return __builtin_nontemporal_load(reinterpret_cast<const d2v*>(a.Qprev + (r < a.nrows ? r : a.nrows - 1) * kB) + li);
      };
      d2v qn = EPI ? qprev_row(0) : d2v{0.0, 0.0};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int64_t r = row_of(blk, k);
        double u0 = acc[k][0], u1 = acc[k][1];
        if constexpr (EPI) {
          const d2v qc = qn;
          if (k < 3) qn = qprev_row(k + 1);
          if (r < a.nrows) {
            double n0 = -qc[0], n1 = -qc[1];
            asm volatile("s_nop 1" : "+v"(n0), "+v"(n1));
            const d2v* bt = reinterpret_cast<const d2v*>(smem + 2 * kPanelBytes);
            pfor<0, 16>([&](auto sc) {
              constexpr int S = decltype(sc)::value;  // u = 2 S (n0 of lane S), 2 S + 1 (n1)
              const d2v be = bt[(2 * S) * 16 + li], bo = bt[(2 * S + 1) * 16 + li];
              pnl_fma<S>(u0, n0, be[0]);
              pnl_fma<S>(u1, n0, be[1]);
              pnl_fma<S>(u0, n1, bo[0]);
              pnl_fma<S>(u1, n1, bo[1]);
            });
          }
        }
        if (r < a.nrows)
          __builtin_nontemporal_store(d2v{u0, u1}, reinterpret_cast<d2v*>(a.U + r * kB) + li);
        acc[k][0] = acc[k][1] = 0.0;
      }
    }
    if (!have_next) break;
    // the next panel's DMA has landed — it is older than the 16 chunk loads just issued, and
    // loads retire in order, so vmcnt(16) leaves those in flight across the barrier — and every
    // wave is done reading this panel (lgkmcnt(0)); a plain __syncthreads() would drain them
    asm volatile("s_waitcnt vmcnt(16)\n\ts_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    buf ^= 1;
    if (last_panel) {
      blk = nblk;
      p0 = np0;
      p1 = np1;
    }
    p = pn;
  }
}

bool spmm_panel(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
                const double* Qprev, const double* Bi, hipStream_t s) {
  if (b != 32 || !A.panel_blk || A.panel_nblk <= 0 || !A.zrow) return false;
  PanelArgs a;
  a.nrows = A.nrows;
  a.nblk = A.panel_nblk;
  a.rowptr = A.rowptr;
  a.col = A.col;
  a.val = A.val;
  a.bpan = A.panel_blk;
  a.Q = Qin;
  a.col_off = col_off;
  a.q_lo = A.q_lo;
  a.q_hi = A.q_hi;
  a.zrow = A.zrow;
  a.U = U;
  a.Qprev = Qprev;
  a.Bi = Bi;
  // one workgroup per CU, a multiple of the 8 XCDs
  const int cus = window_grid();
  const int grid = cus >= pnl::kXcds ? cus / pnl::kXcds * pnl::kXcds : pnl::kXcds;
  if (Qprev) {
    ensure_lds_attr(reinterpret_cast<const void*>(&k_spmm_panel<true>), (int)pnl::kLds);
    hipLaunchKernelGGL(k_spmm_panel<true>, dim3(grid), dim3(pnl::kThreads), pnl::kLds, s, a);
  } else {
    ensure_lds_attr(reinterpret_cast<const void*>(&k_spmm_panel<false>), (int)pnl::kLds);
    hipLaunchKernelGGL(k_spmm_panel<false>, dim3(grid), dim3(pnl::kThreads), pnl::kLds, s, a);
  }
  return true;
}

int panel_rows() { return pnl::kRows; }
int panel_width() { return pnl::kPanel; }

}  // namespace rbl
