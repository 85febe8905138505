// spmm_bt.hip — SpMM over band tiles: the CSR densified ONCE per matrix into 16-row tiles
// stored in v_mfma_f64_4x4x4f64 operand order, streamed from HBM straight into VGPRs.
//
// U = A * Q_i (+ fused 3-term epilogue U -= Q_{i-1} B_i^T, + partials of A_i = Q_i^T U)
//   — RBL_gpu.jl:176-178.
//
// Why: the LDS-densified band kernel (spmm_band.hip) spends its LDS bandwidth twice on A
// (producer zero + scatter of every tile, then every consumer wave re-reading the dense tile)
// and its VALU on the scatter; on gfx950 fp64 MFMA does not co-execute with VALU
// (tools/coexec_probe.hip).  A banded matrix with |c - r| <= H (H = 64 at C4a) fills its
// 16 x (16 + 2H) tile band to 69 % (100 of 144 columns per row), so the densified tile is
// 16*144*8 = 18.4 KB against 16*100*12 = 19.2 KB of CSR values + column indices: storing it
// dense costs no extra HBM and removes the scatter, the column indices and the A traffic
// through LDS altogether.  What stays in LDS is the Q ring (each Q row read from HBM once per
// CU) and, per tile, one ds_read_b128 per (k-step, column pair) of it.
//
// Format (bt_fill): tile t = local rows [16t, 16t+16), band = global columns
// [row0 - H + 16t, row0 + H + 16t + 16) in NG = (2H+16)/16 groups of 16 columns; group g
// holds 2 x 1 KiB: half h, lane l, element s = A[16t + (l&15)][c16 + 16g + 4(2h+s) + (l>>4)]
// — exactly the A operand lane l feeds to the 4x4x4 MFMA of k-step u = 2h+s (layout below),
// one coalesced global_load_dwordx4 per half.
//
// Workgroup: 256 threads = 4 waves, one per SIMD, one workgroup per CU, persistent over a
// contiguous tile range [T0, T1) in rounds of 4 tiles (wave w takes tile T0 + 4r + w).
// Each wave multiplies a whole tile (all 32 columns: 8 accumulators), so A is read once; the
// next tile's group g is loaded into group g's registers as soon as they are consumed (one
// tile period of latency cover, ~18 KiB in flight per wave).  The Q ring (256 rows, in ring
// coordinates rho = global row - (row0 - H)) is filled one round ahead by all four waves
// (register staged), one barrier per round.
//
// v_mfma_f64_4x4x4f64 layout (tools/mfma_layout_probe.hip), block G = (lane>>2)&3:
//   A[row = lane&15][k = lane>>4], B[k = lane>>4][col = lane&3] (same in every block),
//   D[row 4G + (lane>>4)][col lane&3].
// Main product: blocks = the tile's 4 row quads, k = 4 band columns, B = Q ring values.
// Accumulator acc[p][s] column j = lane&3 is U column 8p + 2j + s, so one ds_read_b128 of
// ring row rho at 16-B slot 4p + j feeds acc[p][0] and acc[p][1].
#include <cstdlib>
#include <type_traits>

#include <hipcub/hipcub.hpp>

#include "kernels.hpp"

namespace rbl {

namespace bt {
constexpr int kThreads = 256;
constexpr int kRing = 256;  // ring rows (power of two)
// Geometry per block width B (32 or 16).  Ring row: at B = 32, 16 data slots of 16 B + 4 pad
// slots, so row rho starts at bank slot 4 rho mod 16 and the rows rho, rho+1 (rho+2, rho+3)
// that one ds_read_b128 lane group reads at the same logical slots land on disjoint banks;
// at B = 16 a row is 128 B = 32 banks, so consecutive rows are disjoint already.  U stage row
// (A_i operand): 21 slots at B = 32 (bank shift 5 per row), 128 B at B = 16.
template <int B>
struct Geo {
  static constexpr int kRowBytes = B == 32 ? 320 : 128;
  static constexpr int kRingBytes = kRing * kRowBytes;
  static constexpr int kBtOff = kRingBytes;                  // epilogue B operand table
  static constexpr int kBtBytes = B * B * 8;
  static constexpr int kUStride = B == 32 ? 336 : 128;
  static constexpr int kUWave = 16 * kUStride;
  static constexpr int kUOff = kBtOff + kBtBytes;
  static constexpr int kLds = kUOff + 4 * kUWave;           // B = 32: 111,104 B; B = 16: 43,008 B
  static constexpr int kCtOff = kLds;                       // VAR bit 10: the -C table
  static constexpr int kTrOff = kLds + 9216;                // VAR bit 11: per-wave transpose buffers
  static_assert(kLds + 9216 + 4 * 4 * 2304 <= 160 * 1024, "LDS budget");
};
// A_i operand at B = 32: lane reads ring slot pi(l & 15); pi maps the lanes {0-3, 12-15} of
// each ds_read_b128 lane group to slot classes {0,1} mod 4 and {4-11} to {2,3} mod 4, so rows
// rho (shift 0) and rho+1 (shift 4) never share a bank
__device__ __forceinline__ int pi_slot(int i) {
  const int c = (i >> 2) == 0 ? 0 : (i >> 2) == 1 ? 2 : (i >> 2) == 2 ? 3 : 1;
  return 4 * (i & 3) + c;
}
}  // namespace bt

__device__ __forceinline__ double mfma44(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

struct BtArgs {
  int64_t nrows;
  int64_t ntiles;
  int64_t tiles_per_wg;
  const double* A;       // band tiles (bt_fill)
  const double* Q;       // row c at Q + (c - col_off) * b
  int64_t col_off;
  int64_t q_lo, q_hi;    // global rows present in Q; others read the zero row
  const double* zrow;    // 32 zeros
  const void* Qloc;      // non-null: rows [loc_lo, loc_hi) at Qloc + (c - loc_lo) * b (fp64,
  int64_t loc_lo, loc_hi;  //   or fp32 with VAR bit 6), the rest of [q_lo, q_hi) from Q
  int64_t row0;         // global index of local row 0
  double* U;             // padded to a multiple of 16 rows
  const double* Qprev;
  const float* Q32;      // VAR bit 6: Q and Q_{i-1} are fp32 blocks (the fp32 basis), widened
  const float* Qprev32;  //   exactly on load (RBL_gpu.jl:173-174 copyto!(Qg_d, Qg))
  const double* Bi;
  double* ai_slab;       // AIG: per-workgroup partials of A_i (b x b row-major)
  const uint64_t* hdr;   // VAR bit 7: packed tiles (bt_pack) instead of A
  const double* pv;
  const double* Ah;      // VAR bit 11: half tiles (bt_half) instead of A, and whole tiles for
  const double* Ae;      //   the first NGL local tiles
  const double* Cl;      // VAR bit 10: local reorth on staging (ring rows = Q - Qprev Cl),
  double* Qw;            //   interior own rows written back here (CsrDev::lfix_q); only the
  int64_t lf_lo, lf_hi;  //   local rows [lf_lo, lf_hi) are raw, the others already corrected
};

// ---- local reorth fused into the ring staging (VAR bit 10, B = 32) ----
// Q_i -= Q_{i-1} (Q_{i-1}^T Q_i), one projection (RBL_gpu.jl:83-93, P1), applied to a 16-row
// block as the SpMM stages it: D layout (lane: row 4G + q, columns 8p + 2j + {0, 1}) started
// from the raw rows, then 8 k-steps of 4 MFMAs pairs with A = Q_{i-1} rows (lane & 15, columns
// 8m + 2q + s: the EPI's A layout) and B = -C from an LDS table (row stride kCtLd: the four
// lane groups q read rows 2 apart = 16 banks apart).  k_spmm_bt and k_locfix run this same
// sequence, so a row has the same bits whichever kernel corrects it.
constexpr int kCtLd = 36;
constexpr int kCtBytes = 32 * kCtLd * 8;
constexpr int kTrLd = 18;                  // half tiles: transpose square, doubles per row
constexpr int kTrBytes = 16 * kTrLd * 8;   // per wave (4 x 2,304 B <= 9,216)
// RBL_BT_QNT (diagnostics, default 0): the Q_i / Q_{i-1} rows the SpMM stages load
// non-temporally, so they do not push the half tiles' strips (re-read from L2 by the next
// tiles) out of L2
#ifndef RBL_BT_QNT
#define RBL_BT_QNT 0
#endif
__device__ __forceinline__ d2v qld(const d2v* p) {
  if constexpr (RBL_BT_QNT) return __builtin_nontemporal_load(p);
  return *p;
}
__device__ __forceinline__ void lf_loads(const double* rraw, const double* rprev, int lane,
                                         d2v (&raw)[4], d2v (&qa)[4]) {
  const int q = lane >> 4, j = lane & 3;
#pragma unroll
  for (int p = 0; p < 4; ++p) raw[p] = qld(reinterpret_cast<const d2v*>(rraw + 2 * j) + 4 * p);
#pragma unroll
  for (int m = 0; m < 4; ++m) qa[m] = qld(reinterpret_cast<const d2v*>(rprev + 2 * q) + 4 * m);
}
__device__ __forceinline__ void lf_table(const double* C, double* ct, int tid, int nthreads) {
  for (int idx = tid; idx < 32 * 32; idx += nthreads) ct[(idx >> 5) * kCtLd + (idx & 31)] = -C[idx];
}
__device__ __forceinline__ void lf_block(const d2v (&raw)[4], const d2v (&qa)[4], const double* ct,
                                         int lane, double (&acc)[4][2]) {
  const int q = lane >> 4, j = lane & 3;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    acc[p][0] = raw[p].x;
    acc[p][1] = raw[p].y;
  }
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const double av = s ? qa[m].y : qa[m].x;
      const double* crow = ct + (8 * m + 2 * q + s) * kCtLd + 2 * j;
#pragma unroll
      for (int p = 0; p < 4; ++p) {
        const d2v bv = *reinterpret_cast<const d2v*>(crow + 8 * p);
        acc[p][0] = __builtin_amdgcn_mfma_f64_4x4x4f64(av, bv.x, acc[p][0], 0, 0, 0);
        acc[p][1] = __builtin_amdgcn_mfma_f64_4x4x4f64(av, bv.y, acc[p][1], 0, 0, 0);
      }
    }
}

// VAR: bit 0 non-temporal A loads, bit 1 non-temporal U stores, bit 5 ablation (main-loop
// MFMAs off: loads only), bit 6 fp32 Q / Q_{i-1} inputs, bit 7 packed tiles, bit 8 no LDS
// read-ahead, bit 9 ablation (no round barrier: wrong results, timing only).
//
// Packed tiles: the zeros of the band (31 % at C4a) are not stored.  Per operand block k =
// 2g + h the header holds m0 / m1, bit l = element 0 / 1 of lane l is nonzero, and the block's
// start offset off_k in the tile's value run; lane l's element 0 sits at off_k + mbcnt(m0),
// its element 1 at off_k + popc(m0) + mbcnt(m1), and an absent element is read through a
// buffer load past the run's end, which returns 0.0 — so the MFMA operands, and U, are
// bit-identical to the dense format's.  The masks act directly as lane masks (inverse
// ballot); the tile's header (<= 42 words, one per lane) is loaded one tile ahead of its
// values.
template <int B, int NG, bool EPI, bool AIG, int VAR = 0>
__global__ __launch_bounds__(bt::kThreads) __attribute__((amdgpu_waves_per_eu(1, 1)))
void k_spmm_bt(BtArgs a) {
  using L = bt::Geo<B>;
  constexpr int NP = B / 8;     // U column pairs per lane: acc[p][s] is column 8p + 2j + s
  constexpr int NS = B / 2;     // 16-B slots of a ring row holding data
  constexpr int NE = B / 4;     // epilogue k-steps (Q_{i-1} columns / 4)
  constexpr int H = 8 * (NG - 1);
  constexpr int kRoundRows = 64;                          // 4 tiles
  constexpr int kRingSpan = kRoundRows + 2 * H;           // rows one round reads
  static_assert(kRingSpan + kRoundRows <= bt::kRing, "ring holds a round and the next one's rows");
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t T0 = (int64_t)blockIdx.x * a.tiles_per_wg;
  const int64_t T1 = T0 + a.tiles_per_wg < a.ntiles ? T0 + a.tiles_per_wg : a.ntiles;
  if (T0 >= T1) return;
  const int q = lane >> 4, j = lane & 3, G = (lane >> 2) & 3, i16 = lane & 15;
  const int64_t gq = a.row0 - H;  // global row of ring coordinate 0

  // 16-B chunk (slot s < NS) of the Q row at ring coordinate rho; absent rows read zeros
  auto qload = [&](int64_t rho, int s) -> d2v {
    const int64_t c = rho + gq;
    const bool in = c >= a.q_lo && c < a.q_hi;
    const bool own = c >= a.loc_lo && c < a.loc_hi;  // never when Qloc is null (empty range)
    if constexpr (VAR & 64) {
      const float* p = own ? static_cast<const float*>(a.Qloc) + (c - a.loc_lo) * B
                           : in ? a.Q32 + (c - a.col_off) * B : reinterpret_cast<const float*>(a.zrow);
      const float2 f = reinterpret_cast<const float2*>(p)[s];
      return d2v{(double)f.x, (double)f.y};
    } else {
      const double* p = own ? static_cast<const double*>(a.Qloc) + (c - a.loc_lo) * B
                            : in ? a.Q + (c - a.col_off) * B : a.zrow;
      return qld(reinterpret_cast<const d2v*>(p) + s);
    }
  };
  auto ring_ptr = [&](int64_t rho, int s) -> d2v* {
    return reinterpret_cast<d2v*>(smem + (unsigned)(rho & (bt::kRing - 1)) * L::kRowBytes + 16u * s);
  };

  // ---- prologue: epilogue table, ring rows of round 0 ----
  if constexpr (EPI) {
    // entry ((e*NP + p)*16 + q*4 + j) holds {-B_i[y][x] : s' = 0, 1} with x = 8(e>>1) + 2q +
    // (e&1) (the Q_{i-1} column k-step e feeds), y = 8p + 2j + s'
    double* btab = reinterpret_cast<double*>(smem + L::kBtOff);
    for (int idx = tid; idx < B * B; idx += bt::kThreads) {
      const int sp = idx & 1, jj = (idx >> 1) & 3, qq = (idx >> 3) & 3, p = (idx >> 5) % NP,
                e = (idx >> 5) / NP;
      const int x = 8 * (e >> 1) + 2 * qq + (e & 1), y = 8 * p + 2 * jj + sp;
      btab[idx] = -a.Bi[y * B + x];
    }
  }
  // VAR bit 10: ring rows are staged corrected (local reorth), 16-row blocks per wave
  constexpr bool LF = (VAR & 1024) != 0;
  static_assert(!LF || (B == 32 && !(VAR & (64 | 128))), "fused local reorth: b = 32, fp64, dense tiles");
  double* const ct = reinterpret_cast<double*>(smem + L::kCtOff);
  // written back here: the raw rows of the range's interior (its first and last H rows are
  // read raw by the neighbouring workgroups: k_locfix corrects them after the SpMM)
  const int64_t own_lo = 16 * T0 + H > a.lf_lo ? 16 * T0 + H : a.lf_lo;
  int64_t own_hi = 16 * T1 - H < a.nrows ? 16 * T1 - H : a.nrows;
  own_hi = own_hi < a.lf_hi ? own_hi : a.lf_hi;
  // 16-row block at ring coordinate rho0: rows (D layout) as qload reads them, and the Q_{i-1}
  // rows (A layout) of the raw ones — zero for the rest (rank-edge rows corrected before the
  // halo exchange, neighbours' rows, rows past the matrix), which the MFMAs then leave as read
  auto lf_issue = [&](int64_t rho0, d2v (&raw)[4], d2v (&qa)[4]) {
    const int64_t cr = rho0 + gq + 4 * G + q, ca = rho0 + gq + i16;
    const bool inr = cr >= a.q_lo && cr < a.q_hi;
    const bool ownr = cr >= a.loc_lo && cr < a.loc_hi;  // split halo: own rows from the block
    const int64_t la = ca - a.row0;
    const double* rp = ownr ? static_cast<const double*>(a.Qloc) + (cr - a.loc_lo) * B
                            : inr ? a.Q + (cr - a.col_off) * B : a.zrow;
    lf_loads(rp, la >= a.lf_lo && la < a.lf_hi ? a.Qprev + la * B : a.zrow, lane, raw, qa);
  };
  auto lf_finish = [&](int64_t rho0, const d2v (&raw)[4], const d2v (&qa)[4]) {
    double f[4][2];
    lf_block(raw, qa, ct, lane, f);
    const int64_t rr = rho0 + 4 * G + q;  // ring coordinate of the lane's row
    const int64_t lr = rr + gq - a.row0;  // its local row
    const bool wb = lr >= own_lo && lr < own_hi;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const d2v v = d2v{f[p][0], f[p][1]};
      *ring_ptr(rr, 4 * p + j) = v;
      if (wb) reinterpret_cast<d2v*>(a.Qw + lr * B + 2 * j)[4 * p] = v;
    }
  };
  if constexpr (LF) {
    lf_table(a.Cl, ct, tid, bt::kThreads);
    __syncthreads();
    for (int bb = wave; bb < kRingSpan / 16; bb += 4) {
      d2v raw[4], qa[4];
      lf_issue(16 * T0 + 16 * bb, raw, qa);
      lf_finish(16 * T0 + 16 * bb, raw, qa);
    }
  } else {
    for (int idx = tid; idx < kRingSpan * NS; idx += bt::kThreads) {
      const int64_t rho = 16 * T0 + idx / NS;
      *ring_ptr(rho, idx % NS) = qload(rho, idx % NS);
    }
  }

  // ---- per-wave state ----
  // tiles are stored in consumption order: slot ((round * grid + workgroup) * 4 + wave), so
  // at any moment the whole chip sweeps one contiguous stretch of the format
  const int64_t tslot0 = 4 * (int64_t)blockIdx.x;
  const int64_t tslot_r = 4 * (int64_t)gridDim.x;
  constexpr bool HALF = (VAR & 2048) != 0;
  constexpr int NGL = (NG - 1) / 2, NGH = NG - NGL;  // left groups / stored groups per tile
  static_assert(!HALF || !(VAR & 128), "half tiles are dense");
  // slot of any local tile t (its workgroup's range may be another's): bt_fill's order
  auto slot_of = [&](int64_t t) -> int64_t {
    const int64_t w = t / a.tiles_per_wg, lt = t - w * a.tiles_per_wg;
    return ((lt >> 2) * gridDim.x + w) * 4 + (lt & 3);
  };
  // half tiles: the slots one tile's loads read — its own (groups NGL..NG-1) and, for each left
  // group g, tile t - NGL + g's (its strip group NG-1-g, stored as half group NGL - g) — worked
  // out once per tile, outside the MFMA stream (tile_a is then branch-free); the first NGL
  // local tiles (edge) come whole from Ae
  struct HalfPlan {
    int64_t own = 0;
    int64_t src[NG / 2 > 0 ? NG / 2 : 1] = {};
    bool edge = false;
  };
  auto half_plan = [&](int64_t t) -> HalfPlan {
    HalfPlan hp;
    if constexpr (HALF) {
      const int64_t lt = t - T0;
      hp.own = (lt >> 2) * tslot_r + tslot0 + (lt & 3);
      hp.edge = t < NGL;
      if (!hp.edge) {
#pragma unroll
        for (int g = 0; g < NGL; ++g) {
          const int64_t ls = lt - NGL + g;
          hp.src[g] = ls >= 0 ? (ls >> 2) * tslot_r + tslot0 + (ls & 3) : 0;
        }
        if (lt < NGL) {  // sources before this workgroup's range (rare: division)
#pragma unroll
          for (int g = 0; g < NGL; ++g)
            if (lt - NGL + g < 0) hp.src[g] = slot_of(t - NGL + g);
        }
      }
    }
    return hp;
  };
  auto tile_a = [&](int64_t t, int g, int h, const HalfPlan& hp) -> d2v {
    if constexpr (HALF) {
      const int64_t ts = g >= NGL ? hp.own : hp.src[g < NGL ? g : 0];
      const int gh = g >= NGL ? g - NGL : NGL - g;
      const double* ph = a.Ah + ((((ts * NGH + gh) * 2 + h) * 64) + lane) * 2;
      const double* pe = a.Ae + ((((t * NG + g) * 2 + h) * 64) + lane) * 2;
      const d2v* p = reinterpret_cast<const d2v*>(hp.edge ? pe : ph);
      if constexpr (VAR & 4096) return __builtin_nontemporal_load(p);
      if constexpr (VAR & 1) {
        if (g == NGL) return __builtin_nontemporal_load(p);  // the diagonal group: read once
      }
      return *p;  // strip groups: read again (transposed) by the next NGL tiles — keep in L2
    } else {
      const int64_t lt = t - T0;
      const int64_t ts = (lt >> 2) * tslot_r + tslot0 + (lt & 3);
      const d2v* p = reinterpret_cast<const d2v*>(a.A + ((((ts * NG + g) * 2 + h) * 64) + lane) * 2);
      if constexpr (VAR & 1) return __builtin_nontemporal_load(p);
      return *p;
    }
  };
  // left group g of a half-format tile: lane holds S[r = l & 15][c = 4u + (l >> 4)] of the
  // source strip group (u = 0..3 in v[0].x, v[0].y, v[1].x, v[1].y); the tile needs S^T in the
  // same layout.  Through a wave-private LDS square (row stride kTrLd = 18 doubles: 2-way
  // banked both ways, the minimum for 64 x 8 B).
  // All NGL left groups in one pass (one square each: one LDS round trip per tile), done as soon
  // as the next tile's groups are loaded (end of the current tile), so the reads land while the
  // wave waits at the round barrier.
  auto bt_transpose = [&](d2v (&v)[NG][2]) {
    double* tb0 = reinterpret_cast<double*>(smem + L::kTrOff + wave * NGL * kTrBytes);
#pragma unroll
    for (int g = 0; g < NGL; ++g) {
      double* tb = tb0 + g * (kTrBytes / 8);
      tb[i16 * kTrLd + q] = v[g][0].x;
      tb[i16 * kTrLd + 4 + q] = v[g][0].y;
      tb[i16 * kTrLd + 8 + q] = v[g][1].x;
      tb[i16 * kTrLd + 12 + q] = v[g][1].y;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int g = 0; g < NGL; ++g) {
      const double* tb = tb0 + g * (kTrBytes / 8);
      v[g][0].x = tb[q * kTrLd + i16];
      v[g][0].y = tb[(4 + q) * kTrLd + i16];
      v[g][1].x = tb[(8 + q) * kTrLd + i16];
      v[g][1].y = tb[(12 + q) * kTrLd + i16];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  auto clamp_t = [&](int64_t t) -> int64_t { return t < T1 ? t : T1 - 1; };
  // packed tiles: header words of tile t (lane w holds word w)
  constexpr int PW = bt_pack_words(NG), POFF = 4 * NG, PVB = 4 * NG + (2 * NG + 4) / 4;
  auto hdr_load = [&](int64_t t) -> uint64_t {
    const int64_t lt = t - T0;
    const int64_t ts = (lt >> 2) * tslot_r + tslot0 + (lt & 3);
    return lane < PW ? __builtin_nontemporal_load(a.hdr + ts * PW + lane) : 0ull;
  };
  auto rl32 = [&](uint64_t v, int w, int half) -> unsigned {
    return __builtin_amdgcn_readlane(half ? (unsigned)(v >> 32) : (unsigned)v, w);
  };
  auto rl64 = [&](uint64_t v, int w) -> uint64_t {
    return ((uint64_t)rl32(v, w, 1) << 32) | rl32(v, w, 0);
  };
  auto hoff = [&](uint64_t hd, int k) -> unsigned {  // uint16 k of the offset words
    return (rl32(hd, POFF + (k >> 2), (k >> 1) & 1) >> (16 * (k & 1))) & 0xffffu;
  };
  // lane's two elements of block k = 2g + h of the tile whose run is `rs`: element 0 of
  // lane l at off_k + mbcnt(m0), element 1 at off_k + popc(m0) + mbcnt(m1) (each
  // instruction reads one contiguous stretch); an absent element reads past the run's end,
  // which a buffer load returns as 0.0
  auto tile_ap = [&](uint64_t hd, __amdgpu_buffer_rsrc_t rs, int k) -> d2v {
    const uint64_t m0 = rl64(hd, 2 * k), m1 = rl64(hd, 2 * k + 1);
    const unsigned o = hoff(hd, k);
    unsigned i0 = __builtin_amdgcn_mbcnt_lo((unsigned)m0, o);
    i0 = __builtin_amdgcn_mbcnt_hi((unsigned)(m0 >> 32), i0);
    unsigned i1 = __builtin_amdgcn_mbcnt_lo((unsigned)m1, o + (unsigned)__popcll(m0));
    i1 = __builtin_amdgcn_mbcnt_hi((unsigned)(m1 >> 32), i1);
    const unsigned b0 = __builtin_amdgcn_inverse_ballot_w64(m0) ? 8u * i0 : 0x80000000u;
    const unsigned b1 = __builtin_amdgcn_inverse_ballot_w64(m1) ? 8u * i1 : 0x80000000u;
    return d2v{__builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, b0, 0, 2)),
               __builtin_bit_cast(double, __builtin_amdgcn_raw_buffer_load_b64(rs, b1, 0, 2))};
  };
  auto tile_run = [&](uint64_t hd) -> __amdgpu_buffer_rsrc_t {
    const double* run = a.pv + rl64(hd, PVB);
    return __builtin_amdgcn_make_buffer_rsrc((void*)run, (short)0, (int)(8 * hoff(hd, 2 * NG)),
                                             0x00020000);
  };
  uint64_t hN = 0;  // packed: header of the tile whose values are being loaded
  d2v av[NG][2];
  if constexpr (VAR & 128) {
    const uint64_t h0 = hdr_load(clamp_t(T0 + wave));
    const __amdgpu_buffer_rsrc_t rs = tile_run(h0);
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      av[g][0] = tile_ap(h0, rs, 2 * g);
      av[g][1] = tile_ap(h0, rs, 2 * g + 1);
    }
    hN = hdr_load(clamp_t(T0 + wave + 4));
  } else {
    const HalfPlan hp0 = half_plan(clamp_t(T0 + wave));
#pragma unroll
    for (int g = 0; g < NG; ++g) {
      av[g][0] = tile_a(clamp_t(T0 + wave), g, 0, hp0);
      av[g][1] = tile_a(clamp_t(T0 + wave), g, 1, hp0);
    }
    if constexpr (HALF) {
      if (clamp_t(T0 + wave) >= NGL) bt_transpose(av);
    }
  }
  // Q_{i-1} tile rows: lane row i16, columns 8m + 2q + {0,1}
  auto qprev_load = [&](int64_t t, d2v (&qv)[NE / 2]) {
    int64_t r = 16 * t + i16;
    r = r < a.nrows ? r : a.nrows - 1;
#pragma unroll
    for (int m = 0; m < NE / 2; ++m) {
      if constexpr (VAR & 64) {
        const float2 f = *reinterpret_cast<const float2*>(a.Qprev32 + r * B + 2 * q + 8 * m);
        qv[m] = d2v{(double)f.x, (double)f.y};
      } else {
        qv[m] = reinterpret_cast<const d2v*>(a.Qprev + r * B + 2 * q)[4 * m];
      }
    }
  };
  d2v qp[NE / 2];
  if constexpr (EPI) qprev_load(clamp_t(T0 + wave), qp);
  // A_i accumulators: blocks = 4 x-quads; B = 32: x = 2 pi(4G + q) + xg (xg < 2), B = 16:
  // x = 4G + q; y = 8(yq >> 1) + 2j + (yq & 1)
  constexpr int NXG = B / 16, NYQ = B / 4;
  double ai[NXG][NYQ];
#pragma unroll
  for (int x = 0; x < NXG; ++x)
#pragma unroll
    for (int y = 0; y < NYQ; ++y) ai[x][y] = 0.0;

  const unsigned lb = (unsigned)(q * L::kRowBytes + 16 * j);                // main-loop B
  const unsigned lbt = (unsigned)(L::kBtOff + 16 * (4 * q + j));            // epilogue B
  const unsigned lus = (unsigned)(L::kUOff + wave * L::kUWave);             // U stage
  const unsigned lai = B == 32 ? (unsigned)(16 * bt::pi_slot(i16)) : (unsigned)(8 * i16);
  __syncthreads();

  for (int64_t R = 16 * T0; R < 16 * T1; R += kRoundRows) {
    const int64_t tw = R / 16 + wave;  // this wave's tile
    // ring rows of the next round: 16 per wave (row 4i + q at B = 32, 8i + 2q + (i16 >> 3) at
    // B = 16), slot i16 % NS
    d2v st[4];
    const int64_t rn = R + kRingSpan + 16 * wave;
    auto st_row = [&](int i) -> int64_t {
      return B == 32 ? rn + 4 * i + q : rn + 8 * (i >> 1) + 2 * q + 4 * (i & 1) + (i16 >> 3);
    };
    constexpr int NST = B == 32 ? 4 : 2;
    d2v lraw[4], lqa[4];
    if constexpr (LF) {
      lf_issue(rn, lraw, lqa);
    } else {
#pragma unroll
      for (int i = 0; i < NST; ++i) st[i] = qload(st_row(B == 32 ? i : 2 * i), i16 % NS);
    }

    if (tw < T1) {  // wave-uniform
      const int64_t tn = clamp_t(tw + 4);
      const HalfPlan hpn = half_plan(tn);
      uint64_t hNN = 0;
      if constexpr (VAR & 128) hNN = hdr_load(clamp_t(tw + 8));
      const auto rsN = [&] {
        if constexpr (VAR & 128) return tile_run(hN);
        else return 0;
      }();
      double acc[NP][2];
#pragma unroll
      for (int p = 0; p < NP; ++p) acc[p][0] = acc[p][1] = 0.0;
      // B operands (ring rows) of group g: double-buffered one group ahead, so the ds_reads
      // of group g+1 are in flight while group g's MFMAs issue (one wave per SIMD: nothing
      // else would hide the LDS latency)
      d2v bp[2][4][NP];
      auto ld_bp = [&](int g, d2v (&b)[4][NP]) {
        const unsigned gb = (unsigned)((16 * (tw + g)) & (bt::kRing - 1)) * L::kRowBytes + lb;
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int p = 0; p < NP; ++p)
            b[u][p] = *reinterpret_cast<const d2v*>(smem + gb + u * 4 * L::kRowBytes + 64 * p);
      };
      if constexpr (!(VAR & 256)) ld_bp(0, bp[0]);
#pragma unroll
      for (int g = 0; g < NG; ++g) {
        if constexpr (VAR & 256) ld_bp(g, bp[g & 1]);  // diagnostics: no read-ahead
        else if (g + 1 < NG) ld_bp(g + 1, bp[(g + 1) & 1]);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const double av_u = (u & 1) ? av[g][u >> 1].y : av[g][u >> 1].x;
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            if constexpr (VAR & 32) {  // ablation: loads only (operands consumed, no math)
              asm volatile("" ::"v"(av_u), "v"(bp[g & 1][u][p].x), "v"(bp[g & 1][u][p].y));
            } else {
              acc[p][0] = mfma44(av_u, bp[g & 1][u][p].x, acc[p][0]);
              acc[p][1] = mfma44(av_u, bp[g & 1][u][p].y, acc[p][1]);
            }
          }
        }
        if constexpr (VAR & 128) {  // the next tile's group g into the freed registers
          av[g][0] = tile_ap(hN, rsN, 2 * g);
          av[g][1] = tile_ap(hN, rsN, 2 * g + 1);
        } else {
          av[g][0] = tile_a(tn, g, 0, hpn);
          av[g][1] = tile_a(tn, g, 1, hpn);
        }
      }
      if constexpr (VAR & 128) hN = hNN;
      if constexpr (EPI) {
#pragma unroll
        for (int e = 0; e < NE; ++e) {
          const double qv = (e & 1) ? qp[e >> 1].y : qp[e >> 1].x;
          d2v bv[NP];
#pragma unroll
          for (int p = 0; p < NP; ++p) bv[p] = *reinterpret_cast<const d2v*>(smem + lbt + 256 * (NP * e + p));
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            acc[p][0] = mfma44(qv, bv[p].x, acc[p][0]);
            acc[p][1] = mfma44(qv, bv[p].y, acc[p][1]);
          }
        }
        qprev_load(tn, qp);
      }
      const int64_t ru = 16 * tw + 4 * G + q;  // this lane's U row
      d2v* urow = reinterpret_cast<d2v*>(a.U + ru * B + 2 * j);
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const d2v uv = d2v{acc[p][0], acc[p][1]};
        if constexpr (VAR & 2) __builtin_nontemporal_store(uv, urow + 4 * p);
        else urow[4 * p] = uv;
      }
      if constexpr (AIG) {
        // A_i += Q[tile rows]^T U[tile rows]: blocks = 4 x-quads, k = 4 tile rows, the
        // B operand U[4ks + q][y] shared by the blocks — staged through LDS (D layout in)
        const bool live = ru < a.nrows;
#pragma unroll
        for (int p = 0; p < NP; ++p)
          *reinterpret_cast<d2v*>(smem + lus + (4 * G + q) * L::kUStride + 16 * (4 * p + j)) =
              live ? d2v{acc[p][0], acc[p][1]} : d2v{0.0, 0.0};
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
#pragma unroll
        for (int ks = 0; ks < 4; ++ks) {
          const int64_t rho = 16 * tw + H + 4 * ks + q;  // own rows
          const unsigned rb = (unsigned)(rho & (bt::kRing - 1)) * L::kRowBytes + lai;
          double aq[NXG];
          if constexpr (B == 32) {
            const d2v v = *reinterpret_cast<const d2v*>(smem + rb);
            aq[0] = v.x;
            aq[NXG - 1] = v.y;
          } else {
            aq[0] = *reinterpret_cast<const double*>(smem + rb);
          }
#pragma unroll
          for (int m = 0; m < NYQ / 2; ++m) {
            const d2v bu = *reinterpret_cast<const d2v*>(smem + lus + (4 * ks + q) * L::kUStride + 16 * (4 * m + j));
#pragma unroll
            for (int x = 0; x < NXG; ++x) {
              ai[x][2 * m] = mfma44(aq[x], bu.x, ai[x][2 * m]);
              ai[x][2 * m + 1] = mfma44(aq[x], bu.y, ai[x][2 * m + 1]);
            }
          }
        }
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
        __builtin_amdgcn_wave_barrier();
      }
      if constexpr (HALF) {  // the next tile's left groups, loaded during this tile
        if (tn >= NGL) bt_transpose(av);
      }
    }
    if constexpr (LF) {
      lf_finish(rn, lraw, lqa);
    } else {
#pragma unroll
      for (int i = 0; i < NST; ++i) *ring_ptr(st_row(B == 32 ? i : 2 * i), i16 % NS) = st[i];
    }
    if constexpr (VAR & 512) __builtin_amdgcn_wave_barrier();  // ablation: no round barrier
    else __syncthreads();
  }

  if constexpr (AIG) {
    // sum the 4 waves' partials (ring area, free after the last barrier), wave 0 stores
    double* red = reinterpret_cast<double*>(smem);
    constexpr int NA = NXG * NYQ;
    if (wave > 0) {
#pragma unroll
      for (int x = 0; x < NXG; ++x)
#pragma unroll
        for (int y = 0; y < NYQ; ++y) red[((wave - 1) * NA + x * NYQ + y) * 64 + lane] = ai[x][y];
    }
    __syncthreads();
    if (wave == 0) {
      double* out = a.ai_slab + (int64_t)blockIdx.x * B * B;
      const int xb = B == 32 ? 2 * bt::pi_slot(4 * G + q) : 4 * G + q;
#pragma unroll
      for (int x = 0; x < NXG; ++x)
#pragma unroll
        for (int y = 0; y < NYQ; ++y) {
          double v = ai[x][y];
#pragma unroll
          for (int w = 0; w < 3; ++w) v += red[(w * NA + x * NYQ + y) * 64 + lane];
          out[(xb + x) * B + 8 * (y >> 1) + 2 * j + (y & 1)] = v;
        }
    }
  }
}

#ifdef RBL_VARIANTS
// ---- (variants build only) two waves per SIMD (b = 32, fp64, dense or half tiles) -------------
// measured no faster than k_spmm_bt
// k_spmm_bt holds one wave per SIMD (256 VGPRs + AGPRs), so the SIMD idles whenever that wave
// waits on memory: with whole tiles it streams at the HBM rate anyway, but with half tiles (5.1
// GB less per launch at C4a) it becomes issue-bound at the same time.  Here eight
// waves share one ring: waves p and p + 4 (the same SIMD) split tile T0 + 4r + p by its band
// groups — role 0 the left groups [0, NG0), role 1 the rest — so each holds half the A operands
// and single-buffered B operands (<= 256 registers: two waves per SIMD).  Per round:
//   phase 1  both roles multiply their groups; role 1 leaves its partial U tile in LDS;
//   barrier
//   phase 2  role 0 adds it (U = left part + right part), runs the 3-term epilogue, stores U and
//            forms the A_i partials; role 1 stages the next round's ring rows (with the fused
//            local reorth's 64 MFMAs per 16-row block);
//   barrier.
// The MFMAs per SIMD split ~evenly (role 0: 4 groups + epilogue + A_i, role 1: 5 groups +
// staging at NG = 9).  U differs from k_spmm_bt's only in the association of the group sum.
template <int NG, bool EPI, bool AIG, int VAR>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(2, 2)))
void k_spmm_bt2(BtArgs a) {
  constexpr int B = 32;
  using L = bt::Geo<32>;
  constexpr int NP = 4, NS = 16, NE = 8;
  constexpr int H = 8 * (NG - 1);
  constexpr int kRoundRows = 64;
  constexpr int kRingSpan = kRoundRows + 2 * H;
  static_assert(kRingSpan + kRoundRows <= bt::kRing, "ring");
  constexpr bool LF = (VAR & 1024) != 0, HALF = (VAR & 2048) != 0;
  static_assert(!(VAR & (64 | 128)), "fp64 dense or half tiles");
  constexpr int NGL = (NG - 1) / 2, NGH = NG - NGL;
  constexpr int NG0 = NGL, NG1 = NG - NG0;  // role 0: groups [0, NG0) (the left groups)
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wv = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int p4 = wv & 3, role = wv >> 2;
  const int64_t T0 = (int64_t)blockIdx.x * a.tiles_per_wg;
  const int64_t T1 = T0 + a.tiles_per_wg < a.ntiles ? T0 + a.tiles_per_wg : a.ntiles;
  if (T0 >= T1) return;
  const int q = lane >> 4, j = lane & 3, G = (lane >> 2) & 3, i16 = lane & 15;
  const int64_t gq = a.row0 - H;

  auto qload = [&](int64_t rho, int s) -> d2v {
    const int64_t c = rho + gq;
    const bool in = c >= a.q_lo && c < a.q_hi;
    const bool own = c >= a.loc_lo && c < a.loc_hi;
    const double* p = own ? static_cast<const double*>(a.Qloc) + (c - a.loc_lo) * B
                          : in ? a.Q + (c - a.col_off) * B : a.zrow;
    return qld(reinterpret_cast<const d2v*>(p) + s);
  };
  auto ring_ptr = [&](int64_t rho, int s) -> d2v* {
    return reinterpret_cast<d2v*>(smem + (unsigned)(rho & (bt::kRing - 1)) * L::kRowBytes + 16u * s);
  };
  if constexpr (EPI) {
    double* btab = reinterpret_cast<double*>(smem + L::kBtOff);
    for (int idx = tid; idx < B * B; idx += 512) {
      const int sp = idx & 1, jj = (idx >> 1) & 3, qq = (idx >> 3) & 3, p = (idx >> 5) % NP,
                e = (idx >> 5) / NP;
      const int x = 8 * (e >> 1) + 2 * qq + (e & 1), y = 8 * p + 2 * jj + sp;
      btab[idx] = -a.Bi[y * B + x];
    }
  }
  double* const ct = reinterpret_cast<double*>(smem + L::kCtOff);
  const int64_t own_lo = 16 * T0 + H > a.lf_lo ? 16 * T0 + H : a.lf_lo;
  int64_t own_hi = 16 * T1 - H < a.nrows ? 16 * T1 - H : a.nrows;
  own_hi = own_hi < a.lf_hi ? own_hi : a.lf_hi;
  auto lf_issue = [&](int64_t rho0, d2v (&raw)[4], d2v (&qa)[4]) {
    const int64_t cr = rho0 + gq + 4 * G + q, ca = rho0 + gq + i16;
    const bool inr = cr >= a.q_lo && cr < a.q_hi;
    const bool ownr = cr >= a.loc_lo && cr < a.loc_hi;
    const int64_t la = ca - a.row0;
    const double* rp = ownr ? static_cast<const double*>(a.Qloc) + (cr - a.loc_lo) * B
                            : inr ? a.Q + (cr - a.col_off) * B : a.zrow;
    lf_loads(rp, la >= a.lf_lo && la < a.lf_hi ? a.Qprev + la * B : a.zrow, lane, raw, qa);
  };
  auto lf_finish = [&](int64_t rho0, const d2v (&raw)[4], const d2v (&qa)[4]) {
    double f[4][2];
    lf_block(raw, qa, ct, lane, f);
    const int64_t rr = rho0 + 4 * G + q;
    const int64_t lr = rr + gq - a.row0;
    const bool wb = lr >= own_lo && lr < own_hi;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const d2v v = d2v{f[p][0], f[p][1]};
      *ring_ptr(rr, 4 * p + j) = v;
      if (wb) reinterpret_cast<d2v*>(a.Qw + lr * B + 2 * j)[4 * p] = v;
    }
  };
  if constexpr (LF) {
    lf_table(a.Cl, ct, tid, 512);
    __syncthreads();
    for (int bb = wv; bb < kRingSpan / 16; bb += 8) {
      d2v raw[4], qa[4];
      lf_issue(16 * T0 + 16 * bb, raw, qa);
      lf_finish(16 * T0 + 16 * bb, raw, qa);
    }
  } else {
    for (int idx = tid; idx < kRingSpan * NS; idx += 512) {
      const int64_t rho = 16 * T0 + idx / NS;
      *ring_ptr(rho, idx % NS) = qload(rho, idx % NS);
    }
  }

  const int64_t tslot0 = 4 * (int64_t)blockIdx.x;
  const int64_t tslot_r = 4 * (int64_t)gridDim.x;
  auto slot_of = [&](int64_t t) -> int64_t {
    const int64_t w = t / a.tiles_per_wg, lt = t - w * a.tiles_per_wg;
    return ((lt >> 2) * gridDim.x + w) * 4 + (lt & 3);
  };
  auto lslot = [&](int64_t t) -> int64_t {  // slot of a tile of this workgroup's range
    const int64_t lt = t - T0;
    return (lt >> 2) * tslot_r + tslot0 + (lt & 3);
  };
  // A operands of group g of tile t (whole tiles; half tiles: own groups from the tile's slot,
  // left groups from the strip of tile t - NGL + g, edge tiles whole from Ae)
  auto tile_a = [&](int64_t t, int g, int h) -> d2v {
    if constexpr (HALF) {
      const double* ptr;
      if (t < NGL) {
        ptr = a.Ae + ((((t * NG + g) * 2 + h) * 64) + lane) * 2;
      } else if (g >= NGL) {
        ptr = a.Ah + ((((lslot(t) * NGH + (g - NGL)) * 2 + h) * 64) + lane) * 2;
      } else {
        const int64_t st = t - NGL + g;
        const int64_t ts = st >= T0 ? lslot(st) : slot_of(st);
        ptr = a.Ah + ((((ts * NGH + (NGL - g)) * 2 + h) * 64) + lane) * 2;
      }
      const d2v* p = reinterpret_cast<const d2v*>(ptr);
      if (g == NGL) return __builtin_nontemporal_load(p);  // the diagonal group: read once
      return *p;  // strip groups are read again (transposed) by the next NGL tiles: keep in L2
    } else {
      const d2v* p = reinterpret_cast<const d2v*>(a.A + ((((lslot(t) * NG + g) * 2 + h) * 64) + lane) * 2);
      return __builtin_nontemporal_load(p);
    }
  };
  // half tiles: role 0's NG0 = NGL groups are the left groups, transposed through a wave-private
  // LDS square each (as k_spmm_bt's bt_transpose)
  auto transpose_left = [&](auto& v) {
    double* tb0 = reinterpret_cast<double*>(smem + L::kTrOff + p4 * NGL * kTrBytes);
#pragma unroll
    for (int g = 0; g < NGL; ++g) {
      double* tb = tb0 + g * (kTrBytes / 8);
      tb[i16 * kTrLd + q] = v[g][0].x;
      tb[i16 * kTrLd + 4 + q] = v[g][0].y;
      tb[i16 * kTrLd + 8 + q] = v[g][1].x;
      tb[i16 * kTrLd + 12 + q] = v[g][1].y;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int g = 0; g < NGL; ++g) {
      const double* tb = tb0 + g * (kTrBytes / 8);
      v[g][0].x = tb[q * kTrLd + i16];
      v[g][0].y = tb[(4 + q) * kTrLd + i16];
      v[g][1].x = tb[(8 + q) * kTrLd + i16];
      v[g][1].y = tb[(12 + q) * kTrLd + i16];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  };
  auto clamp_t = [&](int64_t t) -> int64_t { return t < T1 ? t : T1 - 1; };

  auto qprev_load = [&](int64_t t, d2v (&qv)[NE / 2]) {
    int64_t r = 16 * t + i16;
    r = r < a.nrows ? r : a.nrows - 1;
#pragma unroll
    for (int m = 0; m < NE / 2; ++m) qv[m] = reinterpret_cast<const d2v*>(a.Qprev + r * B + 2 * q)[4 * m];
  };
  const unsigned lb = (unsigned)(q * L::kRowBytes + 16 * j);
  const unsigned lbt = (unsigned)(L::kBtOff + 16 * (4 * q + j));
  const unsigned lus = (unsigned)(L::kUOff + p4 * L::kUWave);  // U stage (also the exchange)
  const unsigned lai = (unsigned)(16 * bt::pi_slot(i16));
  constexpr int NXG = 2, NYQ = 8, NA = NXG * NYQ;

  // The two roles run separate copies of the round loop (wave-uniform branch), so each copy's
  // registers hold only its own state: role 0 its 4 left groups, the epilogue operand and the
  // A_i accumulators; role 1 its 5 groups and the staging rows.  Both pass the same barriers.
  auto run = [&](auto role_c) {
    constexpr int R1 = decltype(role_c)::value;
    constexpr int GB = R1 ? NG0 : 0, NGR = R1 ? NG1 : NG0;
    d2v av[NGR][2];
    {
      const int64_t t0 = clamp_t(T0 + p4);
#pragma unroll
      for (int gi = 0; gi < NGR; ++gi) {
        av[gi][0] = tile_a(t0, GB + gi, 0);
        av[gi][1] = tile_a(t0, GB + gi, 1);
      }
      if constexpr (HALF && !R1) {
        if (t0 >= NGL) transpose_left(av);
      }
    }
    d2v qp[NE / 2];
    if constexpr (EPI && !R1) qprev_load(clamp_t(T0 + p4), qp);
    double ai[R1 ? 1 : NXG][R1 ? 1 : NYQ];
    if constexpr (!R1) {
#pragma unroll
      for (int x = 0; x < NXG; ++x)
#pragma unroll
        for (int y = 0; y < NYQ; ++y) ai[x][y] = 0.0;
    }
    __syncthreads();  // the prologue's ring rows and tables

    for (int64_t R = 16 * T0; R < 16 * T1; R += kRoundRows) {
      const int64_t tw = R / 16 + p4;
      const int64_t rn = R + kRingSpan + 16 * p4;  // role 1 stages these 16 rows
      d2v st[R1 && !LF ? 4 : 1], lraw[R1 && LF ? 4 : 1], lqa[R1 && LF ? 4 : 1];
      if constexpr (R1) {
        if constexpr (LF) {
          lf_issue(rn, lraw, lqa);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) st[i] = qload(rn + 4 * i + q, i16);
        }
      }
      const bool live = tw < T1;  // wave-uniform (the same for both roles of a pair)
      const int64_t tn = clamp_t(tw + 4);
      double acc[NP][2];
#pragma unroll
      for (int p = 0; p < NP; ++p) acc[p][0] = acc[p][1] = 0.0;
      // ---- phase 1: this wave's groups ----
      if (live) {
#pragma unroll
        for (int gi = 0; gi < NGR; ++gi) {
          const int g = GB + gi;
          d2v bp[4][NP];
          const unsigned gb = (unsigned)((16 * (tw + g)) & (bt::kRing - 1)) * L::kRowBytes + lb;
#pragma unroll
          for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int p = 0; p < NP; ++p)
              bp[u][p] = *reinterpret_cast<const d2v*>(smem + gb + u * 4 * L::kRowBytes + 64 * p);
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            const double av_u = (u & 1) ? av[gi][u >> 1].y : av[gi][u >> 1].x;
#pragma unroll
            for (int p = 0; p < NP; ++p) {
              acc[p][0] = mfma44(av_u, bp[u][p].x, acc[p][0]);
              acc[p][1] = mfma44(av_u, bp[u][p].y, acc[p][1]);
            }
          }
          av[gi][0] = tile_a(tn, g, 0);
          av[gi][1] = tile_a(tn, g, 1);
        }
      }
      double* xch = reinterpret_cast<double*>(smem + lus);
      if constexpr (R1) {
        if (live) {
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            xch[(2 * p) * 64 + lane] = acc[p][0];
            xch[(2 * p + 1) * 64 + lane] = acc[p][1];
          }
        }
      }
      __syncthreads();
      // ---- phase 2 ----
      if constexpr (!R1) {
        if (live) {
#pragma unroll
          for (int p = 0; p < NP; ++p) {
            acc[p][0] = acc[p][0] + xch[(2 * p) * 64 + lane];
            acc[p][1] = acc[p][1] + xch[(2 * p + 1) * 64 + lane];
          }
          if constexpr (EPI) {
#pragma unroll
            for (int e = 0; e < NE; ++e) {
              const double qv = (e & 1) ? qp[e >> 1].y : qp[e >> 1].x;
              d2v bv[NP];
#pragma unroll
              for (int p = 0; p < NP; ++p) bv[p] = *reinterpret_cast<const d2v*>(smem + lbt + 256 * (NP * e + p));
#pragma unroll
              for (int p = 0; p < NP; ++p) {
                acc[p][0] = mfma44(qv, bv[p].x, acc[p][0]);
                acc[p][1] = mfma44(qv, bv[p].y, acc[p][1]);
              }
            }
            qprev_load(tn, qp);
          }
          const int64_t ru = 16 * tw + 4 * G + q;
          d2v* urow = reinterpret_cast<d2v*>(a.U + ru * B + 2 * j);
#pragma unroll
          for (int p = 0; p < NP; ++p) __builtin_nontemporal_store(d2v{acc[p][0], acc[p][1]}, urow + 4 * p);
          if constexpr (AIG) {
            const bool lv = ru < a.nrows;
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();  // the exchange reads above come before the stage
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int p = 0; p < NP; ++p)
              *reinterpret_cast<d2v*>(smem + lus + (4 * G + q) * L::kUStride + 16 * (4 * p + j)) =
                  lv ? d2v{acc[p][0], acc[p][1]} : d2v{0.0, 0.0};
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
            for (int ks = 0; ks < 4; ++ks) {
              const int64_t rho = 16 * tw + H + 4 * ks + q;
              const unsigned rb = (unsigned)(rho & (bt::kRing - 1)) * L::kRowBytes + lai;
              const d2v v = *reinterpret_cast<const d2v*>(smem + rb);
              const double aq[NXG] = {v.x, v.y};
#pragma unroll
              for (int m = 0; m < NYQ / 2; ++m) {
                const d2v bu = *reinterpret_cast<const d2v*>(smem + lus + (4 * ks + q) * L::kUStride + 16 * (4 * m + j));
#pragma unroll
                for (int x = 0; x < NXG; ++x) {
                  ai[x][2 * m] = mfma44(aq[x], bu.x, ai[x][2 * m]);
                  ai[x][2 * m + 1] = mfma44(aq[x], bu.y, ai[x][2 * m + 1]);
                }
              }
            }
          }
          if constexpr (HALF) {
            if (tn >= NGL) transpose_left(av);
          }
        }
      } else {
        if constexpr (LF) {
          lf_finish(rn, lraw, lqa);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) *ring_ptr(rn + 4 * i + q, i16) = st[i];
        }
      }
      __syncthreads();
    }
    // A_i: the four role-0 waves' partials summed through the (now free) ring area
    double* red = reinterpret_cast<double*>(smem);
    if constexpr (AIG && !R1) {
      if (p4 > 0) {
#pragma unroll
        for (int x = 0; x < NXG; ++x)
#pragma unroll
          for (int y = 0; y < NYQ; ++y) red[((p4 - 1) * NA + x * NYQ + y) * 64 + lane] = ai[x][y];
      }
    }
    __syncthreads();
    if constexpr (AIG && !R1) {
      if (p4 == 0) {
        double* out = a.ai_slab + (int64_t)blockIdx.x * B * B;
        const int xb = 2 * bt::pi_slot(4 * G + q);
#pragma unroll
        for (int x = 0; x < NXG; ++x)
#pragma unroll
          for (int y = 0; y < NYQ; ++y) {
            double v = ai[x][y];
#pragma unroll
            for (int w = 0; w < 3; ++w) v += red[(w * NA + x * NYQ + y) * 64 + lane];
            out[(xb + x) * B + 8 * (y >> 1) + 2 * j + (y & 1)] = v;
          }
      }
    }
  };
  if (role) run(std::integral_constant<int, 1>());
  else run(std::integral_constant<int, 0>());
}

template <int NG, bool EPI, bool AIG, int VAR>
static void launch_bt2_v(const BtArgs& a, int grid, hipStream_t s) {
  constexpr int lds = bt::Geo<32>::kLds + ((VAR & 2048) ? 9216 + 4 * ((NG - 1) / 2) * kTrBytes
                                                       : (VAR & 1024) ? kCtBytes : 0);
  ensure_lds_attr(reinterpret_cast<const void*>(&k_spmm_bt2<NG, EPI, AIG, VAR>), lds);
  hipLaunchKernelGGL((k_spmm_bt2<NG, EPI, AIG, VAR>), dim3(grid), dim3(512), lds, s, a);
}
// RBL_BT2: 1 the two-waves-per-SIMD kernel for b = 32 fp64 steps (EPI + A_i, dense or half
// tiles, with or without the fused local reorth); 0 k_spmm_bt everywhere
static bool bt2_on() {
  const char* e = getenv("RBL_BT2");  // read per launch (tests switch it)
  return e ? atoi(e) != 0 : false;
}
#endif

template <int B, int NG, bool EPI, bool AIG, int VAR>
static void launch_bt_v(const BtArgs& a, int grid, hipStream_t s) {
  constexpr int lds = bt::Geo<B>::kLds + ((VAR & 2048) ? 9216 + 4 * ((NG - 1) / 2) * kTrBytes
                                                      : (VAR & 1024) ? kCtBytes : 0);
  ensure_lds_attr(reinterpret_cast<const void*>(&k_spmm_bt<B, NG, EPI, AIG, VAR>), lds);
  hipLaunchKernelGGL((k_spmm_bt<B, NG, EPI, AIG, VAR>), dim3(grid), dim3(bt::kThreads), lds, s, a);
}
template <int B, int NG, bool EPI, bool AIG>
static void launch_bt_t(const BtArgs& a, int grid, hipStream_t s, bool f32) {
  // default: non-temporal A loads and U stores (VAR 3): the format is read once per launch
  // and U only by the next kernel — measured 7 % faster at C4a than the default policy
#ifndef RBL_VARIANTS
  if (f32) return launch_bt_v<B, NG, EPI, AIG, 3 | 64>(a, grid, s);
  launch_bt_v<B, NG, EPI, AIG, 3>(a, grid, s);
#else
  // RBL_BT_VAR = 0 / 35 / 259 (diagnostics): default policy / loads-only ablation / no LDS
  // read-ahead of the next group's B operands; packed (a.hdr) and half (a.Ah) tiles
  static const int var = [] {
    const char* e = getenv("RBL_BT_VAR");
    return e ? atoi(e) : 3;
  }();
  if (a.hdr) {
    if (f32) return launch_bt_v<B, NG, EPI, AIG, 3 | 64 | 128>(a, grid, s);
    if constexpr (B == 32 && NG == 9 && EPI && AIG) {
      if (var == 35) return launch_bt_v<B, NG, EPI, AIG, 35 | 128>(a, grid, s);
    }
    return launch_bt_v<B, NG, EPI, AIG, 3 | 128>(a, grid, s);
  }
  if (a.Ah) {  // half tiles (bt_half)
    if (f32) return launch_bt_v<B, NG, EPI, AIG, 3 | 64 | 2048>(a, grid, s);
    if constexpr (B == 32 && NG == 9 && EPI && AIG) {  // diagnostics: A load policy
      if (var == 2) return launch_bt_v<B, NG, EPI, AIG, 2 | 2048>(a, grid, s);
      if (var == 4099) return launch_bt_v<B, NG, EPI, AIG, 3 | 2048 | 4096>(a, grid, s);
    }
    return launch_bt_v<B, NG, EPI, AIG, 3 | 2048>(a, grid, s);
  }
  if (f32) return launch_bt_v<B, NG, EPI, AIG, 3 | 64>(a, grid, s);
  if constexpr (B == 32 && NG == 9 && EPI && AIG) {
    if (var == 0) return launch_bt_v<B, NG, EPI, AIG, 0>(a, grid, s);
    if (var == 35) return launch_bt_v<B, NG, EPI, AIG, 35>(a, grid, s);
    if (var == 259) return launch_bt_v<B, NG, EPI, AIG, 259>(a, grid, s);
    if (var == 515) return launch_bt_v<B, NG, EPI, AIG, 515>(a, grid, s);
  }
  launch_bt_v<B, NG, EPI, AIG, 3>(a, grid, s);
#endif
}

bool spmm_bt(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
             const double* Qprev, const double* Bi, hipStream_t s, double* ai_slab, int* ai_parts,
             const float* Q32, const float* Qprev32) {
  if ((b != 32 && b != 16) || !(A.bt || A.bth || A.btp_hdr) || A.ntiles <= 0 || !(A.bt_ng == 5 || A.bt_ng == 9)) return false;
  BtArgs a;
  a.nrows = A.nrows;
  a.ntiles = A.ntiles;
  a.tiles_per_wg = A.bt_tiles_per_wg;
  a.A = A.bt;
  a.Ah = A.bth;
  a.Ae = A.bte;
  a.Q = Qin;
  a.col_off = col_off;
  a.q_lo = A.q_lo;
  a.q_hi = A.q_hi;
  a.zrow = A.zrow;
  a.Qloc = A.qloc;
  a.loc_lo = A.qloc ? A.loc_lo : 0;
  a.loc_hi = A.qloc ? A.loc_hi : 0;
  a.row0 = A.row0;
  a.U = U;
  a.Qprev = Qprev;
  a.Q32 = Q32;
  a.Qprev32 = Qprev32;
  a.Bi = Bi;
  a.hdr = A.btp_hdr;
  a.pv = A.btp_val;
  const int grid = (int)((A.ntiles + A.bt_tiles_per_wg - 1) / A.bt_tiles_per_wg);
  const bool f32 = Q32 != nullptr;
  const bool epi = Qprev != nullptr || Qprev32 != nullptr;
  const bool aig = ai_slab != nullptr;
  a.ai_slab = ai_slab;
  if (ai_parts) *ai_parts = aig ? grid : 0;
  a.Cl = A.lfix_c;
  a.Qw = A.lfix_q;
  if (A.lfix_c) {  // fused local reorth (spmm_bt_locfix_ok checked the format; EPI + A_i here)
    if (b != 32 || f32 || a.hdr || !epi || !aig) return false;
    a.lf_lo = A.lfix_lo;
    a.lf_hi = A.lfix_hi;
#ifdef RBL_VARIANTS
    if (bt2_on()) {
      if (A.two_wave) *A.two_wave = 1;
      if (a.Ah) {
        if (A.bt_ng == 9) launch_bt2_v<9, true, true, 1024 | 2048>(a, grid, s);
        else launch_bt2_v<5, true, true, 1024 | 2048>(a, grid, s);
      } else {
        if (A.bt_ng == 9) launch_bt2_v<9, true, true, 1024>(a, grid, s);
        else launch_bt2_v<5, true, true, 1024>(a, grid, s);
      }
      return true;
    }
    if (a.Ah) {
      if (A.bt_ng == 9) launch_bt_v<32, 9, true, true, 3 | 1024 | 2048>(a, grid, s);
      else launch_bt_v<32, 5, true, true, 3 | 1024 | 2048>(a, grid, s);
      return true;
    }
#endif
    {
      if (A.bt_ng == 9) launch_bt_v<32, 9, true, true, 3 | 1024>(a, grid, s);
      else launch_bt_v<32, 5, true, true, 3 | 1024>(a, grid, s);
    }
    return true;
  }
#ifdef RBL_VARIANTS
  if (bt2_on() && b == 32 && epi && aig && !f32 && !a.hdr) {
    if (A.two_wave) *A.two_wave = 1;
    a.lf_lo = 0;
    a.lf_hi = 0;
    if (a.Ah) {
      if (A.bt_ng == 9) launch_bt2_v<9, true, true, 2048>(a, grid, s);
      else launch_bt2_v<5, true, true, 2048>(a, grid, s);
    } else {
      if (A.bt_ng == 9) launch_bt2_v<9, true, true, 0>(a, grid, s);
      else launch_bt2_v<5, true, true, 0>(a, grid, s);
    }
    return true;
  }
#endif
  const int key = (b == 32 ? 8 : 0) | (A.bt_ng == 9 ? 4 : 0) | (epi ? 2 : 0) | (aig ? 1 : 0);
  switch (key) {
#define RBL_BT_CASE(K, BB, NG, E, G) \
    case K: launch_bt_t<BB, NG, E, G>(a, grid, s, f32); break;
    RBL_BT_CASE(0, 16, 5, false, false) RBL_BT_CASE(1, 16, 5, false, true)
    RBL_BT_CASE(2, 16, 5, true, false)  RBL_BT_CASE(3, 16, 5, true, true)
    RBL_BT_CASE(4, 16, 9, false, false) RBL_BT_CASE(5, 16, 9, false, true)
    RBL_BT_CASE(6, 16, 9, true, false)  RBL_BT_CASE(7, 16, 9, true, true)
    RBL_BT_CASE(8, 32, 5, false, false) RBL_BT_CASE(9, 32, 5, false, true)
    RBL_BT_CASE(10, 32, 5, true, false) RBL_BT_CASE(11, 32, 5, true, true)
    RBL_BT_CASE(12, 32, 9, false, false) RBL_BT_CASE(13, 32, 9, false, true)
    RBL_BT_CASE(14, 32, 9, true, false) RBL_BT_CASE(15, 32, 9, true, true)
#undef RBL_BT_CASE
  }
  return true;
}

// The own rows the fused SpMM left raw (the first and last H rows of each workgroup's tile
// range: its neighbours read them raw as halo), corrected in place after it, one wave per
// 16-row block — the same lf_block sequence, so the same bits as the rows written in the SpMM.
template <int H>
__global__ __launch_bounds__(64) void k_locfix(double* Q, const double* __restrict__ Qprev,
                                               const double* __restrict__ C, int64_t nrows,
                                               int64_t ntiles, int64_t tpw, const double* zrow,
                                               int64_t wlo, int64_t whi) {
  __shared__ __attribute__((aligned(16))) double ct[32 * kCtLd];
  const int lane = threadIdx.x;
  lf_table(C, ct, lane, 64);
  __syncthreads();
  constexpr int per = H / 16;
  const int64_t wg = blockIdx.x / (2 * per);
  const int side = (blockIdx.x / per) & 1, kb = blockIdx.x % per;
  const int64_t T0 = wg * tpw, T1 = T0 + tpw < ntiles ? T0 + tpw : ntiles;
  const int64_t lo = side == 0 ? 16 * T0 : (16 * T0 + H > 16 * T1 - H ? 16 * T0 + H : 16 * T1 - H);
  int64_t hi = side == 0 ? (16 * T1 < 16 * T0 + H ? 16 * T1 : 16 * T0 + H) : 16 * T1;
  hi = hi < nrows ? hi : nrows;
  const int64_t r0 = lo + 16 * kb;
  if (r0 >= hi) return;
  const int q = lane >> 4, j = lane & 3, G = (lane >> 2) & 3, i16 = lane & 15;
  const int64_t rr = r0 + 4 * G + q, ra = r0 + i16;
  d2v raw[4], qa[4];
  lf_loads(rr < nrows ? Q + rr * 32 : zrow, ra < nrows ? Qprev + ra * 32 : zrow, lane, raw, qa);
  double f[4][2];
  lf_block(raw, qa, ct, lane, f);
  if (rr < hi && rr >= wlo && rr < whi) {  // the raw rows only
#pragma unroll
    for (int p = 0; p < 4; ++p) reinterpret_cast<d2v*>(Q + rr * 32 + 2 * j)[4 * p] = d2v{f[p][0], f[p][1]};
  }
}

// Several ranks: the first and last H local rows — the neighbours' halo — corrected in place
// before the halo exchange, so every rank stages them as final rows.  Rows [lo0, hi0) then
// [lo1, hi1), one wave per 16-row block.
__global__ __launch_bounds__(64) void k_locfix_ranges(double* Q, const double* __restrict__ Qprev,
                                                      const double* __restrict__ C, int64_t nrows,
                                                      const double* zrow, int64_t lo0, int64_t hi0,
                                                      int64_t lo1, int64_t hi1) {
  __shared__ __attribute__((aligned(16))) double ct[32 * kCtLd];
  const int lane = threadIdx.x;
  lf_table(C, ct, lane, 64);
  __syncthreads();
  const int64_t nb0 = (hi0 - lo0 + 15) / 16;
  const int64_t r0 = blockIdx.x < nb0 ? lo0 + 16 * (int64_t)blockIdx.x : lo1 + 16 * ((int64_t)blockIdx.x - nb0);
  const int64_t hi = blockIdx.x < nb0 ? hi0 : hi1;
  if (r0 >= hi) return;
  const int q = lane >> 4, j = lane & 3, G = (lane >> 2) & 3, i16 = lane & 15;
  const int64_t rr = r0 + 4 * G + q, ra = r0 + i16;
  d2v raw[4], qa[4];
  lf_loads(rr < nrows ? Q + rr * 32 : zrow, ra < nrows ? Qprev + ra * 32 : zrow, lane, raw, qa);
  double f[4][2];
  lf_block(raw, qa, ct, lane, f);
  if (rr < hi) {
#pragma unroll
    for (int p = 0; p < 4; ++p) reinterpret_cast<d2v*>(Q + rr * 32 + 2 * j)[4 * p] = d2v{f[p][0], f[p][1]};
  }
}

bool spmm_bt_locfix_ok(const CsrDev& A, int b) {
  return b == 32 && (A.bt || A.bth) && !A.btp_hdr && A.ntiles > 0 && (A.bt_ng == 5 || A.bt_ng == 9);
}

int spmm_bt_halfwidth(const CsrDev& A) { return 8 * (A.bt_ng - 1); }

void spmm_bt_locfix_edges(const CsrDev& A, double* Q, const double* Qprev, const double* C,
                          int64_t lo0, int64_t hi0, int64_t lo1, int64_t hi1, hipStream_t s) {
  const int64_t nb = (hi0 - lo0 + 15) / 16 + (hi1 - lo1 + 15) / 16;
  if (nb > 0)
    hipLaunchKernelGGL(k_locfix_ranges, dim3((unsigned)nb), dim3(64), 0, s, Q, Qprev, C, A.nrows, A.zrow,
                       lo0, hi0, lo1, hi1);
}

void spmm_bt_locfix_rest(const CsrDev& A, double* Q, const double* Qprev, const double* C,
                         hipStream_t s) {
  const int64_t grid = (A.ntiles + A.bt_tiles_per_wg - 1) / A.bt_tiles_per_wg;
  if (A.bt_ng == 9)
    hipLaunchKernelGGL(k_locfix<64>, dim3((unsigned)(grid * 8)), dim3(64), 0, s, Q, Qprev, C, A.nrows,
                       A.ntiles, A.bt_tiles_per_wg, A.zrow, A.lfix_lo, A.lfix_hi);
  else
    hipLaunchKernelGGL(k_locfix<32>, dim3((unsigned)(grid * 4)), dim3(64), 0, s, Q, Qprev, C, A.nrows,
                       A.ntiles, A.bt_tiles_per_wg, A.zrow, A.lfix_lo, A.lfix_hi);
}

// ---- format (once per matrix) -----------------------------------------------------------
// Scatter every nonzero (r, c) of the local CSR to its band-tile slot (zero-filled first);
// duplicates add.  One wave per row.
__global__ void k_bt_fill(int64_t nrows, const int64_t* __restrict__ rowptr,
                          const int32_t* __restrict__ col, const double* __restrict__ val,
                          int64_t row0, int H, int NG, int64_t tpw, int64_t grid,
                          double* __restrict__ out) {
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= nrows) return;
  const int64_t t = r >> 4;
  const int64_t wg = t / tpw, lt = t % tpw;
  const int64_t ts = ((lt >> 2) * grid + wg) * 4 + (lt & 3);  // consumption order
  const int i = (int)(r & 15);
  for (int64_t e = rowptr[r] + lane; e < rowptr[r + 1]; e += 64) {
    const int rho = (int)((int64_t)col[e] - (row0 - H) - 16 * t);  // in [0, 16 + 2H)
    const int g = rho >> 4, u = (rho >> 2) & 3, qq = rho & 3;
    const int64_t idx = ((((ts * NG + g) * 2 + (u >> 1)) * 64) + 16 * qq + i) * 2 + (u & 1);
    atomicAdd(out + idx, val[e]);
  }
}

#ifdef RBL_VARIANTS
// (variants build only) Half tiles (A symmetric): tile t's left group g equals the transpose of group NG-1-g of tile
// t - NGL + g bit for bit, so only groups NGL..NG-1 (diagonal + right strip: 10 of 18.4 KB per
// tile at H = 64) are stored and the kernel transposes the strip groups of the previous NGL
// tiles back (L2-resident: read NGL tiles earlier).  U is bit-identical to the whole tiles'.
// k_bt_symcheck: *bad = 1 if any left group of a tile t >= NGL differs from that transpose.
__global__ void k_bt_symcheck(const double* __restrict__ full, int64_t ntiles, int64_t tpw,
                              int64_t grid, int NG, int* bad) {
  const int NGL = (NG - 1) / 2;
  const int64_t per = (int64_t)NGL * 256;
  const int64_t total = (ntiles - NGL) * per;
  auto slot = [&](int64_t t) {
    const int64_t w = t / tpw, lt = t - w * tpw;
    return ((lt >> 2) * grid + w) * 4 + (lt & 3);
  };
  // element (r, c) of group g of the tile in slot ts: lane r + 16 (c & 3), u = c >> 2
  auto at = [&](int64_t ts, int g, int r, int c) {
    const int u = c >> 2;
    return full[((((ts * NG + g) * 2 + (u >> 1)) * 64) + r + 16 * (c & 3)) * 2 + (u & 1)];
  };
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t t = NGL + e / per;
    const int g = (int)((e % per) >> 8), r = (int)(e & 15), c = (int)((e >> 4) & 15);
    const double x = at(slot(t), g, r, c), y = at(slot(t - NGL + g), NG - 1 - g, c, r);
    if (__double_as_longlong(x) != __double_as_longlong(y)) *bad = 1;
  }
}
__global__ void k_bt_half(const double* __restrict__ full, int64_t nslots, int NG,
                          double* __restrict__ half) {
  const int NGL = (NG - 1) / 2, NGH = NG - NGL;
  const int64_t total = nslots * NGH * 256;
  for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t ts = e / (NGH * 256);
    const int64_t rest = e - ts * NGH * 256;
    half[e] = full[(ts * NG + NGL) * 256 + rest];
  }
}

int bt_half(const double* full, int64_t ntiles, int64_t tpw, int NG, double** half,
            double** edge, hipStream_t s) {
  const int64_t grid = (ntiles + tpw - 1) / tpw;
  const int64_t nslots = bt_tile_slots(ntiles, tpw);
  const int NGL = (NG - 1) / 2, NGH = NG - NGL;
  *half = *edge = nullptr;
  int* bad = nullptr;
  if (hipMalloc(&bad, sizeof(int)) != hipSuccess) return (int)hipErrorOutOfMemory;
  int hbad = 0;
  hipMemsetAsync(bad, 0, sizeof(int), s);
  if (ntiles > NGL)
    hipLaunchKernelGGL(k_bt_symcheck, dim3(4096), dim3(256), 0, s, full, ntiles, tpw, grid, NG, bad);
  hipMemcpyAsync(&hbad, bad, sizeof(int), hipMemcpyDeviceToHost, s);
  hipStreamSynchronize(s);
  hipFree(bad);
  if (hbad) return -1;  // not symmetric bit for bit: keep the whole tiles
  if (hipMalloc(half, (size_t)nslots * NGH * 256 * sizeof(double)) != hipSuccess ||
      hipMalloc(edge, (size_t)NGL * NG * 256 * sizeof(double)) != hipSuccess) {
    hipFree(*half);
    *half = nullptr;
    return (int)hipErrorOutOfMemory;
  }
  hipMemsetAsync(*edge, 0, (size_t)NGL * NG * 256 * sizeof(double), s);
  hipLaunchKernelGGL(k_bt_half, dim3(4096), dim3(256), 0, s, full, nslots, NG, *half);
  for (int64_t t = 0; t < NGL && t < ntiles; ++t) {
    const int64_t w = t / tpw, lt = t - w * tpw;
    const int64_t ts = ((lt >> 2) * grid + w) * 4 + (lt & 3);
    hipMemcpyAsync(*edge + t * NG * 256, full + ts * NG * 256, NG * 256 * sizeof(double),
                   hipMemcpyDeviceToDevice, s);
  }
  return (int)hipStreamSynchronize(s);
}

#endif

int64_t bt_tile_slots(int64_t ntiles, int64_t tpw) {
  const int64_t grid = (ntiles + tpw - 1) / tpw;
  return ((tpw + 3) / 4) * grid * 4;
}

void bt_fill(const CsrDev& A, int H, int NG, double* out, hipStream_t s) {
  if (A.nrows <= 0) return;
  const int64_t threads = A.nrows * 64;
  const int64_t tpw = A.bt_tiles_per_wg, grid = (A.ntiles + tpw - 1) / tpw;
  hipLaunchKernelGGL(k_bt_fill, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, A.nrows,
                     A.rowptr, A.col, A.val, A.row0, H, NG, tpw, grid, out);
}

#ifdef RBL_VARIANTS
// (variants build only) Packed tiles (see k_spmm_bt, VAR bit 7): one wave per tile slot.  Pass 1 counts the
// nonzero operand elements, an exclusive scan gives every run's first value, pass 2 writes
// header and run (per block: element 0 of the lanes in lane order, then element 1).
__global__ void k_btp_count(const double* __restrict__ dense, int64_t nslots, int NG,
                            int64_t* __restrict__ cnt) {
  const int64_t ts = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (ts >= nslots) return;
  int64_t c = 0;
  for (int k = 0; k < 2 * NG; ++k) {
    const d2v v = reinterpret_cast<const d2v*>(dense + (ts * 2 * NG + k) * 128)[lane];
    c += __popcll(__ballot(v.x != 0.0)) + __popcll(__ballot(v.y != 0.0));
  }
  if (lane == 0) cnt[ts] = c;
}

__global__ void k_btp_write(const double* __restrict__ dense, int64_t nslots, int NG,
                            const int64_t* __restrict__ vbase, uint64_t* __restrict__ hdr,
                            double* __restrict__ val) {
  const int64_t ts = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (ts >= nslots) return;
  const int PW = bt_pack_words(NG), POFF = 4 * NG, PVB = 4 * NG + (2 * NG + 4) / 4;
  uint64_t* h = hdr + ts * PW;
  uint16_t* offs = reinterpret_cast<uint16_t*>(h + POFF);
  double* run = val + vbase[ts];
  unsigned off = 0;
  for (int k = 0; k < 2 * NG; ++k) {
    const d2v v = reinterpret_cast<const d2v*>(dense + (ts * 2 * NG + k) * 128)[lane];
    const uint64_t m0 = __ballot(v.x != 0.0), m1 = __ballot(v.y != 0.0);
    const unsigned i0 = __builtin_amdgcn_mbcnt_hi((unsigned)(m0 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m0, off));
    const unsigned i1 = __builtin_amdgcn_mbcnt_hi(
        (unsigned)(m1 >> 32), __builtin_amdgcn_mbcnt_lo((unsigned)m1, off + (unsigned)__popcll(m0)));
    if (v.x != 0.0) run[i0] = v.x;
    if (v.y != 0.0) run[i1] = v.y;
    if (lane == 0) {
      h[2 * k] = m0;
      h[2 * k + 1] = m1;
      offs[k] = (uint16_t)off;
    }
    off += (unsigned)(__popcll(m0) + __popcll(m1));
  }
  if (lane == 0) {
    offs[2 * NG] = (uint16_t)off;
    h[PVB] = (uint64_t)vbase[ts];
  }
}

int bt_pack(const double* dense, int64_t nslots, int NG, uint64_t* hdr, double** val_out,
            int64_t* nval_out, hipStream_t s) {
  *val_out = nullptr;
  *nval_out = 0;
  if (nslots <= 0) return 0;
  int64_t *cnt = nullptr, *vb = nullptr;
  void* tmp = nullptr;
  size_t tb = 0;
  hipError_t e = hipMalloc(&cnt, (nslots + 1) * sizeof(int64_t));
  if (e == hipSuccess) e = hipMalloc(&vb, (nslots + 1) * sizeof(int64_t));
  const unsigned blocks = (unsigned)((nslots * 64 + 255) / 256);
  if (e == hipSuccess) e = hipMemsetAsync(cnt, 0, (nslots + 1) * sizeof(int64_t), s);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_btp_count, dim3(blocks), dim3(256), 0, s, dense, nslots, NG, cnt);
    e = hipcub::DeviceScan::ExclusiveSum(nullptr, tb, cnt, vb, (int)(nslots + 1), s);
  }
  if (e == hipSuccess) e = hipMalloc(&tmp, tb);
  if (e == hipSuccess) e = hipcub::DeviceScan::ExclusiveSum(tmp, tb, cnt, vb, (int)(nslots + 1), s);
  int64_t total = 0;
  if (e == hipSuccess) e = hipMemcpyAsync(&total, vb + nslots, sizeof(int64_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  if (e == hipSuccess) e = hipMalloc(val_out, total * sizeof(double));
  if (e == hipSuccess) e = hipMemsetAsync(hdr, 0, nslots * bt_pack_words(NG) * sizeof(uint64_t), s);
  if (e == hipSuccess) {
    hipLaunchKernelGGL(k_btp_write, dim3(blocks), dim3(256), 0, s, dense, nslots, NG, vb, hdr, *val_out);
    e = hipGetLastError();
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(tmp);
  (void)hipFree(cnt);
  (void)hipFree(vb);
  if (e != hipSuccess) {
    (void)hipFree(*val_out);
    *val_out = nullptr;
    return (int)e;
  }
  *nval_out = total;
  return 0;
}

#endif

}  // namespace rbl
