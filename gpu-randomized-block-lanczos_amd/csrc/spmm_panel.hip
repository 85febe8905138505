// spmm_panel.hip — column-panel SpMM for wide bands (gfx950), b = 32, fp64.
//
// U = A * Q_i  (+ the 3-term epilogue U -= Q_{i-1} B_i^T), RBL_gpu.jl:176-177, for matrices
// whose rows reach further than the band-tile (|c - r| <= 64) and LDS-window (a 256-row ring)
// kernels allow — the FEM / circuit orderings of the reference's benchmark.jl:21-28 inputs,
// bandwidths in the hundreds to thousands.  HBM-bound: SURVEY §8(d) prices a launch at
// nnz * (8 + 4) + (n + 1) * 8 + n * b * 8 * (2 + EPI) bytes; this kernel streams nnz * (8 + 1)
// record bytes plus the Q panels each row block stages.
//
// A workgroup (1024 threads, one per CU, persistent) owns row blocks of R = 64 RPG rows.  A
// block's columns span [cmin, cmax]; that window is walked in column panels of kPanel = 256 Q
// rows (64 KiB at b = 32), double-buffered in LDS and filled by LDS-DMA
// (global_load_lds_dwordx4): while panel p is multiplied the next one streams into the other
// buffer, and one barrier per panel swaps them.  A Q row is read from L2 / HBM once per block
// and then from LDS once per nonzero (the 256 B per nonzero are the kernel's main on-chip
// traffic: ds_read_b128).  R trades registers for staging: the panels cost (R + 2H) / R Q
// blocks of traffic per launch.
//
// The format (panel_format, built once per matrix): within a block the CSR records are
// regrouped panel-major — panel by panel, and within a panel row by row, each row's entries in
// column order (so a row's sum within a panel runs in the CSR's order) — with the column stored as one
// byte, its offset in the panel.  A step (block, panel) therefore reads one contiguous run of
// records, and no cache line is fetched by two steps; per row and panel the format holds the
// count (uint16) and the first record (uint32 from the block's base).
//
//   * rows: 16-lane group G = tid / 16 (64 per workgroup) owns rows G + 64 k (k < RPG) of the
//     block; lane li holds columns 2 li, 2 li + 1 of each row's accumulator
//   * a row's records in panel p: CH per load (more in a loop) — the next step's right after the
//     row's entries in this one, into the same registers; count and start two steps ahead.
//     Lanes past the count load out of range (buffer loads: no traffic, value 0, column 0), so
//     they multiply panel row 0 by zero with no mask
//   * per entry: v_add_u32_dpp forms the Q row's LDS address from the broadcast offset
//     (row_newbcast), one ds_read_b128, and two v_fmac_f64_dpp with the broadcast value; the
//     four groups of a wave step through their rows' counts together (the wave loops to the
//     largest)
//   * hipcc drains an in-flight LDS-DMA at the first use of any ordinary load's result, so a
//     step first touches everything the step before loaded, then issues its DMA and the loads
//     for the next steps; the barrier waits for the DMA with a counted vmcnt, leaving those in
//     flight
//   * the epilogue (B_i^T as a per-lane LDS table, Q_{i-1} rows one ahead) and the store of U
//     end a block.
// Work goes to the workgroups XCD by XCD: the 8 XCDs take contiguous eighths of the blocks and
// an XCD's 32 workgroups sweep theirs side by side, so neighbouring blocks — whose windows
// overlap by 2H rows — read shared panels close together in time (L2 / Infinity Cache).  A
// block walks its window's np panels from the one = 0 (mod np), wrapping round (kOrder 1): the
// workgroups, in near lockstep, then read panels of one residue at each step — the same few
// panels at the same time — instead of panels two steps apart (-2 % at H = 256..2048,
// profiles/r06_panel_v9_order_ab_b24.txt).  A row's sum thus runs panel by panel in that
// rotated order (deterministic; the window and gather kernels keep the CSR's order).
#include <cstdint>
#include <type_traits>
#include <utility>

#include "kernels.hpp"

namespace rbl {

namespace pnl {
constexpr int kThreads = 1024;
constexpr int kGroups = 64;                      // 16-lane row groups per workgroup
constexpr int kPanel = 256;                      // Q rows per panel
constexpr int kB = 32;
constexpr int kRowBytes = kB * 8;                // 256
constexpr int kPanelBytes = kPanel * kRowBytes;  // 64 KiB
constexpr int kBtBytes = kB * 16 * 16;           // B_i^T table: [u][lane] double2
constexpr size_t kLds = 2 * (size_t)kPanelBytes + kBtBytes;
constexpr int kXcds = 8;
constexpr unsigned kOob = 0x10000000u;           // a record offset past any block's records
// probe builds only (-DRBL_PANEL_ABLATE=mask, tools/build_variant.sh): 1 no FMAs, 2 no LDS
// reads, 4 no panel DMA, 8 no record loads — wrong results, for timing what each part costs
#ifndef RBL_PANEL_ABLATE
#define RBL_PANEL_ABLATE 0
#endif
constexpr int kAbl = RBL_PANEL_ABLATE;
// the order a block walks its panels: 1 (default) residue-aligned — step pi of a block reads the
// panel of its window that is = pi (mod np), so the XCD's workgroups, which step through their
// blocks in near lockstep, read the same few panels at the same time (L2 serves the re-reads);
// 0 ascending from the window's first panel (probe builds, for A/B)
#ifndef RBL_PANEL_ORDER
#define RBL_PANEL_ORDER 1
#endif
constexpr int kOrder = RBL_PANEL_ORDER;
// probe builds only (-DRBL_PANEL_STAMPS=1): workgroups 0 and 128 print the cycles their wave 0
// spent in each phase of the step loop (s_memtime), once per launch
#ifndef RBL_PANEL_STAMPS
#define RBL_PANEL_STAMPS 0
#endif
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
// x from lane S of the lane's 16-lane row (after the 2 wait states a VALU-written x needs)
template <int S>
__device__ __forceinline__ int pnl_bcast(int x) {
  int r;
  asm("s_nop 1\n\tv_mov_b32_dpp %0, %1 row_newbcast:%2 row_mask:0xf bank_mask:0xf"
      : "=v"(r) : "v"(x), "n"(S));
  return r;
}
// the panel row at off (from lane S of the lane's 16-lane row) + lane_off: ds_read_b128 issued as
// inline asm, so the compiler neither sinks it into the branch that uses it nor waits for it —
// the caller waits (lgkmcnt) and keeps the destination live until then
template <int S>
__device__ __forceinline__ void pnl_read(double __attribute__((ext_vector_type(2)))& q, unsigned off,
                                         unsigned lane_off) {
  asm volatile("ds_read_b128 %0, %1" : "=v"(q) : "v"(pnl_addr<S>(off, lane_off)));
}
// make the compiler wait for a loaded register here (no instruction)
__device__ __forceinline__ void touch(int x) { asm volatile("" ::"v"(x)); }
__device__ __forceinline__ void touch(double x) { asm volatile("" ::"v"(x)); }

}  // namespace

struct PanelArgs {
  int64_t nrows;             // local rows
  int64_t nblk;              // blocks of 64 RPG rows
  const int64_t* rowptr;     // a block's base: rowptr[b R]
  const uint8_t* pcol;       // the panel-major records: column within the panel
  const double* pval;        //   and value
  const int32_t* binfo;      // per block: first panel, last panel, count offset (2 x int32)
  const uint16_t* cnt;       // per block and panel of its window: R counts (entries per row)
  const uint32_t* st;        // ... and R first records (from the block's base)
  const double* Q;           // Q row c at Q + (c - col_off) * 32, rows [q_lo, q_hi)
  int64_t col_off, q_lo, q_hi;
  const double* zrow;        // >= 32 zeros: the panel rows outside [q_lo, q_hi)
  double* U;
  const double* Qprev;       // may be null (no epilogue)
  const double* Bi;          // b x b row-major (B_i), with Qprev
};

template <bool EPI, int RPG, int CH>
__global__ __launch_bounds__(pnl::kThreads) void k_spmm_panel(PanelArgs a) {
  using namespace pnl;
  constexpr int R = kGroups * RPG;
  constexpr int NCR = CH / 16;  // chunk registers per row
  static_assert(CH % 16 == 0 && CH <= 64, "chunks of 16 to 64 entries per row");
  constexpr int kVm = 2 * NCR * RPG;  // chunk loads per step (the barrier's vmcnt)
  constexpr int QW = RPG == 8 ? 2 : 4;  // LDS reads per group in flight ahead (registers)
  constexpr int NQ = 16 / QW;
  typedef double d2v __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) unsigned char lds_u8;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int li = lane & 15;
  const int grp = tid >> 4;  // 0..63
  const int wave = tid >> 6;

  // ---- this workgroup's blocks: XCD x (= blockIdx % 8) takes blocks [x nblk / 8, (x+1) nblk / 8)
  // and its workgroups j = blockIdx / 8 take every (gridDim / 8)-th of them ----
  const int nper = gridDim.x / kXcds;
  const int xcd = blockIdx.x % kXcds, j = blockIdx.x / kXcds;
  const int64_t xb1 = a.nblk * (xcd + 1) / kXcds;
  const int64_t blk0 = a.nblk * xcd / kXcds + j;
  if (blk0 >= xb1) return;  // whole workgroup: uniform

  if constexpr (EPI) {  // B_i^T as a per-lane table: bt[u][l] = (B_i[2l][u], B_i[2l+1][u])
    d2v* bt = reinterpret_cast<d2v*>(smem + 2 * kPanelBytes);
    for (int e = tid; e < kB * 16; e += kThreads) {
      const int u = e >> 4, l = e & 15;
      bt[e] = d2v{a.Bi[(2 * l) * kB + u], a.Bi[(2 * l + 1) * kB + u]};
    }
  }
  const unsigned lds_base = (unsigned)(size_t)(lds_u8*)smem;
  const unsigned lane_off = (unsigned)(li * 16);

  // ---- block-uniform values through the scalar cache (read-only here) ----
  typedef __attribute__((address_space(4))) const int64_t c_i64;
  typedef __attribute__((address_space(4))) const int32_t c_i32;
  c_i64* rp_s = (c_i64*)a.rowptr;
  c_i32* bi_s = (c_i32*)a.binfo;

  // a step of the workgroup's sweep: (block, panel index within the block's window)
  struct Step {
    int64_t blk;
    int pi, np, p0;  // step index within the block, panels of the block, its first panel (global id)
    int o;           // the window's panel of step 0 (residue order): step pi takes (pi + o) mod np
    int64_t coff;    // the block's counts
  };
  // the panel (index within the block's window) that step s multiplies
  auto win_panel = [&](const Step& s) -> int {
    if constexpr (kOrder == 0) return s.pi;
    const int w = s.pi + s.o;
    return w >= s.np ? w - s.np : w;
  };
  auto block_step = [&](int64_t b) -> Step {
    Step s;
    s.blk = b;
    s.pi = 0;
    s.p0 = s.np = 0;
    s.coff = 0;
    s.o = 0;
    if (b < xb1) {
      s.p0 = bi_s[4 * b];
      s.np = bi_s[4 * b + 1] - s.p0 + 1;
      s.coff = (int64_t)(uint32_t)bi_s[4 * b + 2] | ((int64_t)bi_s[4 * b + 3] << 32);
      if constexpr (kOrder == 1) {  // p0 + o = 0 (mod np)
        const int r = s.p0 % s.np;
        s.o = r == 0 ? 0 : s.np - (r < 0 ? r + s.np : r);
      }
    }
    return s;
  };
  auto next_step = [&](const Step& s) -> Step {
    if (s.blk < xb1 && s.pi + 1 < s.np) {
      Step t = s;
      ++t.pi;
      return t;
    }
    return block_step(s.blk < xb1 ? s.blk + nper : s.blk);
  };
  auto block_base = [&](int64_t b) -> int64_t {
    const int64_t r = b * R;
    return rp_s[r < a.nrows ? r : a.nrows];
  };
  auto rsrc_of = [&](int64_t b, __amdgpu_buffer_rsrc_t& rc, __amdgpu_buffer_rsrc_t& rv) {
    const int64_t z0 = block_base(b), z1 = block_base(b + 1);
    const int64_t n = z1 - z0;
    rc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.pcol + z0), 0, (int)n, 0x00020000);
    rv = __builtin_amdgcn_make_buffer_rsrc(const_cast<double*>(a.pval + z0), 0, (int)(n * 8), 0x00020000);
  };

  // ---- panel staging: LDS-DMA, no staging registers.  Wave w's instruction i writes 1 KiB =
  // rows 4 (w + 16 i) .. + 3 of the panel (lane l: row + l / 16, bytes 16 (l % 16)); rows
  // outside [q_lo, q_hi) come from a zero row ----
  auto load_panel = [&](int p, int buf) {
    const int64_t cb0 = (int64_t)p * kPanel;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int rl = 4 * (wave + 16 * i);
      const int64_t c = cb0 + rl + (lane >> 4);
      const double* src = (c >= a.q_lo && c < a.q_hi) ? a.Q + (c - a.col_off) * kB + 2 * li
                                                      : a.zrow + 2 * li;
      if constexpr (!(kAbl & 4))
        __builtin_amdgcn_global_load_lds(src, smem + buf * kPanelBytes + rl * kRowBytes, 16, 0, 0);
    }
  };
  // records [c0, c0 + min(m, CH)) of a row into chunk registers (lane li: c0 + li, + 16);
  // lanes past m load nothing (an offset past the block's records reads 0)
  auto load_chunk = [&](int (&cc)[NCR], double (&vv)[NCR], int c0, int m, __amdgpu_buffer_rsrc_t rc,
                        __amdgpu_buffer_rsrc_t rv) {
#pragma unroll
    for (int r = 0; r < NCR; ++r) {
      const int e = 16 * r + li;
      const unsigned o = e < m ? (unsigned)(c0 + e) : kOob;
      if constexpr (kAbl & 8) {
        cc[r] = (int)(o & 0xff);
        vv[r] = 0.0;
      } else {
        cc[r] = __builtin_amdgcn_raw_buffer_load_b8(rc, (int)o, 0, 0);
        vv[r] = __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rv, (int)(o * 8u), 0, 0));
      }
    }
  };
  // a step's counts and first records: lane li < RPG holds row k = li's (rows past the slice
  // were counted 0)
  auto load_cs = [&](const Step& s, int& m, int& c0) {
    m = c0 = 0;
    if (s.blk >= xb1 || li >= RPG) return;
    const int64_t i = s.coff + (int64_t)win_panel(s) * R + grp + 64 * li;
    m = a.cnt[i];
    c0 = (int)a.st[i];
  };

  double acc[RPG][2];
  int cc[RPG][NCR];         // each row's chunk: the current step's records, then the next's
  double vv[RPG][NCR];
#pragma unroll
  for (int k = 0; k < RPG; ++k) acc[k][0] = acc[k][1] = 0.0;

  // ---- prologue: step 0's counts, starts, chunks and panel; step 1's counts and starts ----
  Step st = block_step(blk0);
  Step st1 = next_step(st);
  __amdgpu_buffer_rsrc_t rc, rv;
  rsrc_of(blk0, rc, rv);
  int cnt_cur, s_cur;
  load_cs(st, cnt_cur, s_cur);
  pfor<0, RPG>([&](auto kc) {
    constexpr int k = decltype(kc)::value;
    load_chunk(cc[k], vv[k], pnl_bcast<k>(s_cur), pnl_bcast<k>(cnt_cur), rc, rv);
  });
  int cnt_nxt, s_nxt;
  load_cs(st1, cnt_nxt, s_nxt);
  load_panel(st.p0 + win_panel(st), 0);
  __syncthreads();  // (drains everything: the prologue's loads and DMA)

  int buf = 0;
#if RBL_PANEL_STAMPS
  uint64_t ph[6] = {0, 0, 0, 0, 0, 0};
  uint64_t tp = __builtin_readcyclecounter();
  int nsteps = 0;
  auto stamp = [&](int i) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    const uint64_t t = __builtin_readcyclecounter();
    ph[i] += t - tp;
    tp = t;
  };
#define PNL_STAMP(i) stamp(i)
#else
#define PNL_STAMP(i) ((void)0)
#endif
  for (;;) {
    const bool last_panel = st.pi + 1 == st.np;
    const Step sn = st1;
    const bool have_next = sn.blk < xb1;
    const Step sn2 = next_step(sn);
    const unsigned bufb = lds_base + (unsigned)(buf * kPanelBytes);

    // (1) everything the step before loaded, waited for here — before this step's DMA
#pragma unroll
    for (int k = 0; k < RPG; ++k) {
#pragma unroll
      for (int r = 0; r < NCR; ++r) {
        touch(cc[k][r]);
        touch(vv[k][r]);
      }
    }
    touch(cnt_cur);
    touch(s_cur);
    touch(cnt_nxt);
    touch(s_nxt);
    __builtin_amdgcn_sched_barrier(0);

    PNL_STAMP(0);
    // (2) the next step's panel, then the loads the next steps need (younger than the DMA)
    if (have_next) load_panel(sn.p0 + win_panel(sn), buf ^ 1);
    asm volatile("" ::: "memory");
    int cnt_nn = 0, s_nn = 0;
    if (have_next) load_cs(sn2, cnt_nn, s_nn);
    // where the next step's chunks come from: this block, or the next one
    __amdgpu_buffer_rsrc_t rcn = rc, rvn = rv;
    if (have_next && last_panel) rsrc_of(sn.blk, rcn, rvn);
    // the epilogue's Q_{i-1} rows, loaded here where registers allow (4 rows per group): their
    // latency then runs under the step's multiply instead of before the epilogue's FMAs
    // Issued on every step (from the zero row unless the block ends here) as inline asm: hipcc
    // would wait vmcnt(0) for an ordinary load behind the in-flight DMA, draining the next
    // step's record loads; the epilogue waits vmcnt(kVm) for these itself (the record loads of
    // (3), kVm of them, are the only younger vector-memory ops; the "memory" clobbers keep them
    // on their side of both asm statements).  Not with 48-record chunks: their registers
    // (128 VGPRs without these; 64 B of scratch with them).
    constexpr bool kQpEarly = EPI && RPG == 4 && CH <= 32;
    d2v qpe[kQpEarly ? RPG : 1];
    if constexpr (kQpEarly) {
#pragma unroll
      for (int k = 0; k < RPG; ++k) {
        const int64_t r = st.blk * R + grp + 64 * k;
        const double* src = last_panel ? a.Qprev + (r < a.nrows ? r : a.nrows - 1) * kB + 2 * li : a.zrow;
        asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(qpe[k]) : "v"(src) : "memory");
      }
    }

    PNL_STAMP(1);
    // lane k (< RPG) of every group: the largest count of row k over the wave's four groups
    int cmax4 = max(cnt_cur, __shfl_xor(cnt_cur, 16));
    cmax4 = max(cmax4, __shfl_xor(cmax4, 32));
    // (3) multiply the panel, row by row; each row's chunk for the next step follows its entries
    pfor<0, RPG>([&](auto kc) {
      constexpr int k = decltype(kc)::value;
      const int m = pnl_bcast<k>(cnt_cur);  // this group's row k: entries in the panel
      const int mmax = __builtin_amdgcn_readlane(cmax4, k);  // the wave's largest (uniform)
      double& a0 = acc[k][0];
      double& a1 = acc[k][1];
      // QW entries QW J .. QW J + QW - 1 of one chunk register: their LDS reads, issued one group
      // ahead of their FMAs (a group's reads are in flight while the group before is multiplied)
      auto readg = [&](d2v (&q)[QW], unsigned off, auto jc) {
        constexpr int J = decltype(jc)::value;
        pfor<0, QW>([&](auto ic) {
          constexpr int S = QW * J + decltype(ic)::value;
          if constexpr (kAbl & 2) {
            q[decltype(ic)::value] = d2v{(double)pnl_addr<S>(off, lane_off), 0.0};
          } else {
            pnl_read<S>(q[decltype(ic)::value], off, lane_off);
          }
        });
      };
      auto fmag = [&](const d2v (&q)[QW], double w, auto jc) {
        constexpr int J = decltype(jc)::value;
        pfor<0, QW>([&](auto ic) {
          constexpr int S = QW * J + decltype(ic)::value;
          if constexpr (kAbl & 1) {
            touch(q[decltype(ic)::value][0]);
            touch(q[decltype(ic)::value][1]);
          } else {
            pnl_fma<S>(a0, w, q[decltype(ic)::value][0]);
            pnl_fma<S>(a1, w, q[decltype(ic)::value][1]);
          }
        });
      };
      // wait until at most N LDS reads are in flight; q's registers count as written here
      auto waitg = [&](d2v (&q)[QW], auto nc) {
        constexpr int N = decltype(nc)::value;
        if constexpr (QW == 2) asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(q[0]), "+v"(q[1]) : "n"(N));
        else asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(q[0]), "+v"(q[1]), "+v"(q[2]), "+v"(q[3]) : "n"(N));
      };
      auto run = [&](int done) {
        unsigned u[NCR];
        double x[NCR];
#pragma unroll
        for (int r = 0; r < NCR; ++r) {  // lanes past the count: column 0, value 0 (loaded)
          u[r] = bufb + ((unsigned)cc[k][r] << 8);
          x[r] = vv[k][r];
        }
        // VALU write -> DPP read needs 2 wait states; hipcc does not pad inside asm
        if constexpr (NCR == 1) asm volatile("s_nop 1" : "+v"(u[0]), "+v"(x[0]));
        if constexpr (NCR == 2) asm volatile("s_nop 1" : "+v"(u[0]), "+v"(u[1]), "+v"(x[0]), "+v"(x[1]));
        if constexpr (NCR == 3)
          asm volatile("s_nop 1" : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(x[0]), "+v"(x[1]), "+v"(x[2]));
        if constexpr (NCR == 4)
          asm volatile("s_nop 1" : "+v"(u[0]), "+v"(u[1]), "+v"(u[2]), "+v"(u[3]), "+v"(x[0]), "+v"(x[1]),
                       "+v"(x[2]), "+v"(x[3]));
        const int left = mmax - done;
        // the wave's groups of QW entries (uniform branches): a group's reads are issued while
        // the group before is multiplied, and lgkmcnt(QW) then waits for the older group only.
        // The read-ahead is unconditional inside a taken group (past the count it reads panel
        // row 0: harmless) — a read issued on one path only would leave its registers to a
        // merge the compiler may resolve with a copy made before the data lands
        pfor<0, NCR>([&](auto rr) {
          constexpr int RR = decltype(rr)::value;
          if (16 * RR < left) {
            d2v qa[QW], qb[QW];
            readg(qa, u[RR], std::integral_constant<int, 0>{});
            pfor<0, NQ>([&](auto jc) {
              constexpr int J = decltype(jc)::value;
              if (16 * RR + QW * J < left) {
                d2v(&cur)[QW] = J % 2 == 0 ? qa : qb;
                d2v(&nxt)[QW] = J % 2 == 0 ? qb : qa;
                if constexpr (J + 1 < NQ) {
                  readg(nxt, u[RR], std::integral_constant<int, J + 1>{});
                  waitg(cur, std::integral_constant<int, QW>{});
                } else {
                  waitg(cur, std::integral_constant<int, 0>{});
                }
                fmag(cur, x[RR], jc);
              }
            });
            // the read-ahead past the last group taken may still be landing in qa / qb: wait for
            // it while both are live (the compiler must not reuse their registers before)
            if constexpr (QW == 2)
              asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(qa[0]), "+v"(qa[1]), "+v"(qb[0]), "+v"(qb[1]));
            else
              asm volatile("s_waitcnt lgkmcnt(0)" : "+v"(qa[0]), "+v"(qa[1]), "+v"(qa[2]), "+v"(qa[3]),
                           "+v"(qb[0]), "+v"(qb[1]), "+v"(qb[2]), "+v"(qb[3]));
          }
        });
      };
      run(0);
      // more than CH entries in this panel in some group: the next CH, loaded here (rare
      // when CH covers the typical count)
      for (int done = CH; done < mmax; done += CH) {
        load_chunk(cc[k], vv[k], pnl_bcast<k>(s_cur) + done, m - done, rc, rv);
        run(done);
      }
      // the next step's records of this row (past the last step the count is 0: every lane
      // out of range — issued anyway, so the loads' order is the same on every path)
      load_chunk(cc[k], vv[k], pnl_bcast<k>(s_nxt), pnl_bcast<k>(cnt_nxt), rcn, rvn);
    });

    PNL_STAMP(2);
    // (4) block end: epilogue, store U.  Q_{i-1} rows are loaded four at a time, and B_i^T's
    // table is read once per four rows (two LDS reads per u pair), whose FMAs are independent;
    // each row's sum runs in the same order as one row at a time
    if (last_panel) {
      if constexpr (EPI) {
        constexpr int EH = RPG < 4 ? RPG : 4;  // rows per pass (registers)
        pfor<0, RPG / EH>([&](auto hc) {
          constexpr int K0 = EH * decltype(hc)::value;
          d2v qn[EH];  // -Q_{i-1} rows: all loads first, then the negations (one wait)
#pragma unroll
          for (int k = 0; k < EH; ++k) {
            if constexpr (kQpEarly) {
              if (k == 0)  // (the loads of (2): wait here, tied to their registers)
                asm volatile("s_waitcnt vmcnt(%4)" : "+v"(qpe[0]), "+v"(qpe[1]), "+v"(qpe[2]), "+v"(qpe[3])
                             : "n"(kVm) : "memory");
              qn[k] = qpe[K0 + k];
            } else {
              const int64_t r = st.blk * R + grp + 64 * (K0 + k);
              qn[k] = *(reinterpret_cast<const d2v*>(a.Qprev + (r < a.nrows ? r : a.nrows - 1) * kB) + li);
            }
          }
#pragma unroll
          for (int k = 0; k < EH; ++k) {
            qn[k] = -qn[k];
            asm volatile("s_nop 1" : "+v"(qn[k]));
          }
          const d2v* bt = reinterpret_cast<const d2v*>(smem + 2 * kPanelBytes);
          pfor<0, 16>([&](auto sc) {
            constexpr int S = decltype(sc)::value;  // u = 2 S (qn[.][0] of lane S), 2 S + 1 ([1])
            const d2v be = bt[(2 * S) * 16 + li], bo = bt[(2 * S + 1) * 16 + li];
#pragma unroll
            for (int k = 0; k < EH; ++k) {
              pnl_fma<S>(acc[K0 + k][0], qn[k][0], be[0]);
              pnl_fma<S>(acc[K0 + k][1], qn[k][0], be[1]);
              pnl_fma<S>(acc[K0 + k][0], qn[k][1], bo[0]);
              pnl_fma<S>(acc[K0 + k][1], qn[k][1], bo[1]);
            }
          });
        });
      }
#pragma unroll
      for (int k = 0; k < RPG; ++k) {
        const int64_t r = st.blk * R + grp + 64 * k;
        if (r < a.nrows)
          __builtin_nontemporal_store(d2v{acc[k][0], acc[k][1]}, reinterpret_cast<d2v*>(a.U + r * kB) + li);
        acc[k][0] = acc[k][1] = 0.0;
      }
    }
    PNL_STAMP(3);
#if RBL_PANEL_STAMPS
    ++nsteps;
#endif
    if (!have_next) break;
    // (5) the DMA has landed — older than the step's other loads, which retire in order, so a
    // counted vmcnt leaves those (at least the kVm chunk loads) in flight across the barrier —
    // and every wave is done reading this panel (lgkmcnt(0)).  A plain __syncthreads() would
    // drain them.
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_waitcnt lgkmcnt(0)" ::"n"(kVm) : "memory");
    PNL_STAMP(4);
    __builtin_amdgcn_s_barrier();
    PNL_STAMP(5);
    buf ^= 1;
    rc = rcn;
    rv = rvn;
    cnt_cur = cnt_nxt;
    s_cur = s_nxt;
    cnt_nxt = cnt_nn;
    s_nxt = s_nn;
    st = sn;
    st1 = sn2;
  }
#if RBL_PANEL_STAMPS
  if ((blockIdx.x == 0 || blockIdx.x == 128) && tid == 0)
    printf("panel stamps wg %d steps %d: touch %llu issue %llu compute %llu epi %llu vmwait %llu barrier %llu\n",
           (int)blockIdx.x, nsteps, (unsigned long long)ph[0], (unsigned long long)ph[1],
           (unsigned long long)ph[2], (unsigned long long)ph[3], (unsigned long long)ph[4],
           (unsigned long long)ph[5]);
#endif
}

// RPG / CH by the format's mean count per row and panel (rbl_api.cpp, prepare_window_formats):
// <8, 16> up to 16, <4, 48> beyond (<8, 32> needs more than 128 VGPRs with the quad read-ahead;
// <4, 48> against <4, 32>: a row's ~25-50 entries per panel at half-widths 128-512 in one chunk
// instead of a chunk and a reload, 0.5-2.4 % faster, profiles/r06_panel_shapes_b30.txt)
bool spmm_panel(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
                const double* Qprev, const double* Bi, hipStream_t s) {
  if (b != 32 || !A.panel_blk || A.panel_nblk <= 0 || !A.panel_cnt || !A.panel_st || !A.panel_col ||
      !A.panel_val || !A.zrow)
    return false;
  PanelArgs a;
  a.nrows = A.nrows;
  a.nblk = A.panel_nblk;
  a.rowptr = A.rowptr;
  a.pcol = A.panel_col;
  a.pval = A.panel_val;
  a.binfo = A.panel_blk;
  a.cnt = A.panel_cnt;
  a.st = A.panel_st;
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
  auto go = [&](auto kern) {
    ensure_lds_attr(reinterpret_cast<const void*>(kern), (int)pnl::kLds);
    hipLaunchKernelGGL(kern, dim3(grid), dim3(pnl::kThreads), pnl::kLds, s, a);
  };
#ifdef RBL_PANEL_RPG  // (probe builds: one shape for every matrix)
  if (Qprev) go(&k_spmm_panel<true, RBL_PANEL_RPG, RBL_PANEL_CH>);
  else go(&k_spmm_panel<false, RBL_PANEL_RPG, RBL_PANEL_CH>);
  return true;
#endif
  if (A.panel_rpg == 8) {
    if (Qprev) go(&k_spmm_panel<true, 8, 16>); else go(&k_spmm_panel<false, 8, 16>);
  } else {
    if (Qprev) go(&k_spmm_panel<true, 4, 48>); else go(&k_spmm_panel<false, 4, 48>);
  }
  return true;
}

int panel_width() { return pnl::kPanel; }

// ---- the format.  Per block of R rows: its panel range and count offset (binfo, host-made);
// the count of every row's entries in every panel of the range (cnt, zero-filled first); their
// first records, an exclusive scan of the block's counts in (panel, row) order (st); the
// records regrouped in that order (pcol / pval) ----
__global__ void k_panel_counts(int64_t nrows, const int64_t* __restrict__ rowptr,
                               const int32_t* __restrict__ col, const int32_t* __restrict__ binfo,
                               int R, uint16_t* __restrict__ cnt) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  const int64_t b = r / R;
  const int p0 = binfo[4 * b];
  const int64_t coff = (int64_t)(uint32_t)binfo[4 * b + 2] | ((int64_t)binfo[4 * b + 3] << 32);
  const int rl = (int)(r - b * R);
  int pc = -1, n = 0;
  for (int64_t e = rowptr[r]; e < rowptr[r + 1]; ++e) {
    const int p = col[e] / pnl::kPanel;
    if (p != pc) {
      if (pc >= 0) cnt[coff + (int64_t)(pc - p0) * R + rl] = (uint16_t)n;
      pc = p;
      n = 0;
    }
    ++n;
  }
  if (pc >= 0) cnt[coff + (int64_t)(pc - p0) * R + rl] = (uint16_t)n;
}

// one workgroup (256 threads) per block: the exclusive scan of its counts, 256 at a time
__global__ __launch_bounds__(256) void k_panel_starts(const int32_t* __restrict__ binfo, int R,
                                                      const uint16_t* __restrict__ cnt,
                                                      uint32_t* __restrict__ st) {
  __shared__ uint32_t wsum[4];
  const int64_t b = blockIdx.x;
  const int np = binfo[4 * b + 1] - binfo[4 * b] + 1;
  const int64_t coff = (int64_t)(uint32_t)binfo[4 * b + 2] | ((int64_t)binfo[4 * b + 3] << 32);
  const int64_t len = (int64_t)np * R;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t carry = 0;
  for (int64_t i0 = 0; i0 < len; i0 += 256) {
    const int64_t i = i0 + threadIdx.x;
    const uint32_t v = i < len ? cnt[coff + i] : 0u;
    uint32_t x = v;  // inclusive scan within the wave
#pragma unroll
    for (int d = 1; d < 64; d <<= 1) {
      const uint32_t y = __shfl_up(x, d, 64);
      if (lane >= d) x += y;
    }
    if (lane == 63) wsum[w] = x;
    __syncthreads();
    uint32_t before = carry;
    for (int k = 0; k < w; ++k) before += wsum[k];
    const uint32_t total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
    if (i < len) st[coff + i] = before + x - v;
    carry += total;
    __syncthreads();
  }
}

__global__ void k_panel_scatter(int64_t nrows, const int64_t* __restrict__ rowptr,
                                const int32_t* __restrict__ col, const double* __restrict__ val,
                                const int32_t* __restrict__ binfo, int R,
                                const uint32_t* __restrict__ st, uint8_t* __restrict__ pcol,
                                double* __restrict__ pval) {
  const int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (r >= nrows) return;
  const int64_t b = r / R;
  const int p0 = binfo[4 * b];
  const int64_t coff = (int64_t)(uint32_t)binfo[4 * b + 2] | ((int64_t)binfo[4 * b + 3] << 32);
  const int rl = (int)(r - b * R);
  const int64_t zb = rowptr[b * R];
  int pc = -1;
  int64_t o = 0;
  for (int64_t e = rowptr[r]; e < rowptr[r + 1]; ++e) {
    const int c = col[e];
    const int p = c / pnl::kPanel;
    if (p != pc) {
      pc = p;
      o = zb + st[coff + (int64_t)(p - p0) * R + rl];
    }
    pcol[o] = (uint8_t)(c - p * pnl::kPanel);
    pval[o] = val[e];
    ++o;
  }
}

int panel_format(const CsrDev& A, const int32_t* binfo, int R, int64_t nblk, uint16_t* cnt,
                 uint32_t* st, int64_t ncnt, uint8_t* pcol, double* pval, hipStream_t s) {
  if (hipMemsetAsync(cnt, 0, (size_t)ncnt * sizeof(uint16_t), s) != hipSuccess) return -1;
  if (A.nrows > 0) {
    const dim3 g((unsigned)((A.nrows + 255) / 256));
    hipLaunchKernelGGL(k_panel_counts, g, dim3(256), 0, s, A.nrows, A.rowptr, A.col, binfo, R, cnt);
    hipLaunchKernelGGL(k_panel_starts, dim3((unsigned)nblk), dim3(256), 0, s, binfo, R, cnt, st);
    hipLaunchKernelGGL(k_panel_scatter, g, dim3(256), 0, s, A.nrows, A.rowptr, A.col, A.val, binfo,
                       R, st, pcol, pval);
  }
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace rbl
