// spmm_band.hip — persistent CSR SpMM for banded sparsity with the band tile densified in
// LDS and multiplied on fp64 MFMA (gfx950).
//
// U = A * Q_i (+ fused 3-term epilogue U -= Q_{i-1} B_i^T) — RBL_gpu.jl:176-177.
// HBM traffic is exactly the CSR stream (nnz*(8+4) + (n+1)*8) plus Q_i, Q_{i-1} and U once.
//
// Why densify: a row-per-nonzero kernel (spmm_window.hip) reads one b*8-byte Q row from LDS
// per nonzero; at n=1e7, nnz=1e9, b=32 that is 256 GB of LDS reads — as long as the whole
// HBM stream.  Here each 16-row tile's band (columns [cmin, cmax], <= 160 wide) is scattered
// from CSR into a dense LDS tile and multiplied with the Q ring rows by v_mfma_f64_4x4x4f64:
// every Q ring row is read once per tile (not once per nonzero).  The zero fill costs flops
// (16 x K dense vs nnz), which the MFMA pipe absorbs while HBM stays the bound.
//
// Workgroup: 1024 threads (16 waves), one per CU, persistent over a contiguous tile range,
// split by role (the phase stamps of RBL_SPMM_PROF showed that one role doing both, compute
// then staging behind a per-tile barrier, serialises the two: ~6000 cycles per tile):
//   * waves 8..15 produce: in phase t they move the register-staged data of tile t+2 into
//     LDS (zero + scatter two dense rows per wave, the tile's new Q ring rows, its Q_{i-1}
//     rows) and issue the global loads of tile t+2+kRegStages.  Loads are SGPR-base +
//     lane-offset, 16 B per lane for the CSR stream, and unconditional (col/val padded by
//     kCsrPad, row indices clamped; lanes past a row re-read its last group): each stage
//     issues a fixed set of VMEM ops, so vmcnt waits count only the stage consumed.
//   * waves 0..7 consume: in phase t they multiply tile t — wave c owns column group
//     cg = c % (b/4) (and k-half h = c / (b/4) at b=16) over the band, four accumulators
//     (the dependent 4x4x4 f64 MFMA chain is 44 cycles), A operands two k-steps per
//     ds_read_b128 (perm8 column order), B operands from the Q ring at a running byte address
//     (+4 rows per k-step, masked to the ring size) — then the fused 3-term epilogue and the
//     store of 16 x 4 of U (at b=16 the k-halves meet in LDS one phase later).
//   Both roles run their own loop with one barrier per tile; dense tiles, Q_{i-1} tiles and
//   tile descriptors are triple-buffered (compute t, staged t+1, being written t+2).
// v_mfma_f64_4x4x4f64 layout (tools/mfma_layout_probe.hip), block g = (lane>>2)&3 on row
// quad g: A[row = lane&15][k = lane>>4], B[k = lane>>4][col = lane&3], D[row 4g + (lane>>4)][lane&3].
#include <cstdio>
#include <cstdlib>

#include "kernels.hpp"

namespace rbl {

namespace band {
constexpr int kTileRows = 16;
constexpr int kThreads = 1024;
constexpr int kConsumers = 8;         // waves 0..7
constexpr int kProducers = 8;         // waves 8..15, two tile rows each
constexpr int kMaxK = 160;            // band width per tile (columns)
// dense tile rows: columns stored at perm8(k) so a lane's k-steps u, u+1 (columns k, k+4)
// come in one ds_read_b128; the 16 rows of a lane group land on distinct 16-B bank slots
// when kAdLd = 4 mod 32 (slot(r, q) = 2r + q mod 16 over each group's (r, q) set).
// Positions kMaxK.. are never read by compute: kTrash is the scatter's discard slot.
constexpr int kAdLd = kMaxK + 4;
constexpr int kTrash = kMaxK;
constexpr int kRing = 256;            // ring rows (power of two: byte addresses wrap by mask)
constexpr int kBufs = 3;
static_assert(perm8(kTrash) == kTrash && kTrash + 1 < kAdLd, "trash slot layout");
static_assert((kConsumers + kProducers) * 64 == kThreads && 2 * kProducers == kTileRows,
              "roles: 8 consumer waves, 8 producer waves of two tile rows");
}  // namespace band
// CSR entries: a producer lane holds entries 4l..4l+3 of a row counted from the row start
// rounded down to a multiple of 4 (16-B aligned col / 32-B aligned val loads): rows of up to
// 253 nonzeros in one int4 + two double2 loads per lane.

__device__ __forceinline__ double mfma4b(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

struct BandArgs {
  int64_t nrows;
  int64_t ntiles;
  int64_t tiles_per_wg;
  const int64_t* rowptr;
  const int32_t* col;    // padded by kCsrPad entries
  const double* val;     // padded by kCsrPad entries
  const int64_t* tinfo;  // per tile: e0, nnz, lo, hi, cmin, cmax, 0, 0
  const double* Q;       // rows [col_off, ...) of the halo-extended Q
  int64_t col_off;
  double* U;             // padded to a multiple of 16 rows
  const double* Qprev;
  const double* Bi;
  double* ai_slab;           // AIG: per-workgroup partials of A_i = Q[own rows]^T U (b x b)
  int64_t row0;              // global index of local row 0 (ring rows are global)
  int ablate;                // diagnostics only (RBL_SPMM_ABLATE=1: skip compute)
  unsigned long long* prof;  // diagnostics only (PROF instantiation)
};

template <int B>
struct BandLayout {
  static constexpr int NCG = B / 4;                   // column groups of 4
  static constexpr int KSPLIT = band::kConsumers / NCG;  // consumer waves per column group
  // ring row = B doubles, no padding: at b=32 the two rows a 32-lane half reads in one
  // ds_read_b64 (q = 0/1 or 2/3) would share banks, so column c of ring row r is stored at
  // c ^ ((r & 1) << 2) (4 columns = 8 banks apart); at b=16 rows r, r+1 are 32 banks apart.
  static constexpr int kSwz = B == 32 ? 4 : 0;
  static constexpr int kRowBytes = B * 8;
  static constexpr int kRingBytes = band::kRing * kRowBytes;   // 64 KiB / 32 KiB
  static constexpr int QPLD = 36;              // Q_{i-1} tile stride, = 4 mod 32 (as kAdLd)
  static constexpr int kAdOff = kRingBytes;
  static constexpr int kAdBytes = band::kTileRows * band::kAdLd * 8;
  static constexpr int kQpOff = kAdOff + band::kBufs * kAdBytes;
  static constexpr int kQpBytes = band::kTileRows * QPLD * 8;
  static constexpr int kXchOff = kQpOff + band::kBufs * kQpBytes;
  static constexpr int kXchBytes = (KSPLIT - 1) * NCG * 64 * 8;
  static constexpr int kDescOff = kXchOff + 2 * kXchBytes;
  static constexpr int kLds = kDescOff + band::kBufs * 16;
  static_assert(kLds <= 160 * 1024, "LDS budget");
};

struct BandRow {
  int cnt;    // entries of the row
  int shift;  // row start - 4-aligned start (0..3)
  int4 c;
  d2v v0, v1;
};

// PAIR staging: the two rows of a producer wave are contiguous in CSR, so one set of 16-B
// lane loads (64 lanes x 4 entries) covers both when their nonzeros + alignment shift fit 256
// (checked on the host: CsrDev::band_pair); r0 then holds the pair and r1 is unused.
struct BandStage {
  int64_t desc_next;  // lane l <= 16: rowptr[16T'+l]; 17..20: lo, hi, cmin, cmax of the next tile
  int nnew, lo, cmin, K;  // of the tile the registers below hold (wave-uniform)
  int cnt0;               // PAIR: entries of the first row of the pair
  BandRow r0, r1;
  double q0, q1;      // new ring rows, two elements per producer thread
  double qp;          // Q_{i-1} tile, one element per producer thread
};

__device__ __forceinline__ int lane32(int64_t v, int l) {
  return __builtin_amdgcn_readlane((int)(v & 0xffffffffll), l);
}

// PROF (diagnostic instantiation, RBL_SPMM_PROF=1): per-wave shader-clock cycles of work
// and of barrier wait, summed into a.prof[wave * 4 + {0,1,3}] (3 = tiles).
// AIG: the consumers also form A_i = Q^T U over the tile rows (RBL_gpu.jl:178) while U is
// in registers: in the MFMA D layout a lane holds U[4g + (lane>>4)][4cg + (lane&3)], which
// is the B operand (B[k][j] = U[4g+k][4cg+j]) of the 4x4x4 MFMA whose A operand is the
// ring element Q[4g + (lane>>4)][4qc + (lane&3)] (A[i][k] = Q[4g+k][4qc+i]); block g yields
// the row quad's share of (Q^T U)[4qc+i][4cg+j], summed over blocks at the end.
template <int B, bool EPI, bool PROF = false, bool AIG = false, bool PAIR = false>
__global__ __launch_bounds__(band::kThreads) void k_spmm_band(BandArgs a) {
  using L = BandLayout<B>;
  constexpr int NCG = L::NCG, KSPLIT = L::KSPLIT, QPLD = L::QPLD;
  constexpr int EKS = (B / 4) / KSPLIT;  // epilogue k-steps per consumer wave
  constexpr int kRegStages = 3;          // register sets of prefetched tile data
  constexpr unsigned kRingMask = L::kRingBytes - 1;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  auto adb = [&](int buf) { return reinterpret_cast<double*>(smem + L::kAdOff + buf * L::kAdBytes); };
  auto qpb = [&](int buf) { return reinterpret_cast<double*>(smem + L::kQpOff + buf * L::kQpBytes); };
  auto xcb = [&](int buf) { return reinterpret_cast<double*>(smem + L::kXchOff + buf * L::kXchBytes); };
  auto dsb = [&](int buf) { return reinterpret_cast<int*>(smem + L::kDescOff + buf * 16); };

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int64_t t0 = (int64_t)blockIdx.x * a.tiles_per_wg;
  const int64_t t1 = t0 + a.tiles_per_wg < a.ntiles ? t0 + a.tiles_per_wg : a.ntiles;
  if (t0 >= t1) return;

  auto ring_addr = [&](int row, int col) -> unsigned {  // byte address of a Q ring element
    return ((unsigned)(row & (band::kRing - 1)) * L::kRowBytes) +
           (unsigned)((col ^ ((row & 1) ? L::kSwz : 0)) * 8);
  };
  // one lane-vector load per tile descriptor (clamped addresses: always issued)
  auto load_desc = [&](int64_t t) -> int64_t {
    const int64_t tc = t < t1 ? t : t1 - 1;
    const int64_t r = tc * band::kTileRows + lane;
    const int64_t* p = lane <= 16 ? a.rowptr + (r < a.nrows ? r : a.nrows)
                                  : a.tinfo + tc * 8 + 2 + (lane <= 20 ? lane - 17 : 0);
    return *p;
  };

  unsigned long long pw = 0, pb = 0, px = 0;
  auto stamp = [&]() -> unsigned long long {
    if constexpr (PROF) return __builtin_amdgcn_s_memtime();
    return 0;
  };

  // ---- prologue: the first tile's ring window, by every thread ----
  for (int i = tid; i < L::kRingBytes / 8; i += band::kThreads) reinterpret_cast<double*>(smem)[i] = 0.0;
  __syncthreads();
  {
    const int64_t d0 = load_desc(t0);
    const int cmin0 = lane32(d0, 19), cmax0 = lane32(d0, 20);
    for (int e = tid; e < (cmax0 - cmin0 + 1) * B; e += band::kThreads) {
      const int row = cmin0 + e / B, col = e % B;
      *reinterpret_cast<double*>(smem + ring_addr(row, col)) = a.Q[(int64_t)(row - a.col_off) * B + col];
    }
  }

  if (wave >= band::kConsumers) {
    // =============================== producers ===============================
    const int p = wave - band::kConsumers;     // tile rows 2p, 2p+1
    const int ptid = tid - band::kConsumers * 64;
    constexpr int kQStep = 512 / B;             // rows between a thread's two ring elements
    const int qr = ptid / B, qc = ptid % B;
    const int qp_off = qr * QPLD + perm8(qc);   // qr < 16 for the threads that store Q_{i-1}
    constexpr int kQpWaves = band::kTileRows * B / 64;  // producer waves storing Q_{i-1}

    auto load_row = [&](int64_t rs, int cnt, BandRow& R) {
      R.cnt = cnt;
      R.shift = (int)(rs & 3);
      const int ng = (cnt + R.shift + 3) >> 2;
      const int l = lane < ng ? lane : (ng > 0 ? ng - 1 : 0);
      const int32_t* cb = a.col + (rs - R.shift);
      const double* vb = a.val + (rs - R.shift);
      R.c = reinterpret_cast<const int4*>(cb)[l];
      R.v0 = reinterpret_cast<const d2v*>(vb)[2 * l];
      R.v1 = reinterpret_cast<const d2v*>(vb)[2 * l + 1];
    };
    // take the descriptor loaded kRegStages phases ago, issue tile t's loads and the
    // descriptor load of tile t + kRegStages
    auto load_stage = [&](int64_t t, BandStage& S) {
      const int rs_lo = lane32(S.desc_next, 2 * p);
      const int rs_hi = __builtin_amdgcn_readlane((int)(S.desc_next >> 32), 2 * p);
      const int64_t rs = ((int64_t)rs_hi << 32) | (unsigned)rs_lo;
      const int m_lo = lane32(S.desc_next, 2 * p + 1), e_lo = lane32(S.desc_next, 2 * p + 2);
      const int lo = lane32(S.desc_next, 17), hi = lane32(S.desc_next, 18);
      S.cmin = lane32(S.desc_next, 19);
      S.K = lane32(S.desc_next, 20) - S.cmin + 1;
      S.lo = lo;
      S.nnew = hi - lo;
      S.desc_next = load_desc(t + kRegStages);
      if constexpr (PAIR) {
        S.cnt0 = m_lo - rs_lo;
        load_row(rs, e_lo - rs_lo, S.r0);  // both rows: one load set
      } else {
        load_row(rs, m_lo - rs_lo, S.r0);
        load_row(rs + (m_lo - rs_lo), e_lo - m_lo, S.r1);
      }
      // new ring rows lo + qr and lo + qr + kQStep, clamped to the last new row (threads
      // past it re-read and later re-store that row's data)
      const int nq = S.nnew > 0 ? S.nnew : 1;
      const int qrow0 = (S.nnew > 0 ? lo : S.cmin) - (int)a.col_off;  // a valid row of Qin
      const double* qb = a.Q + (int64_t)qrow0 * B;
      const int l0 = qr < nq ? qr : nq - 1, l1 = qr + kQStep < nq ? qr + kQStep : nq - 1;
      S.q0 = qb[l0 * B + qc];
      S.q1 = qb[l1 * B + qc];
      if constexpr (EPI) {
        const int64_t tc = t < t1 ? t : t1 - 1;
        const int64_t last = a.nrows - 1 - tc * band::kTileRows;  // >= 0
        const int prc = qr < last ? qr : (int)last;
        const int off = p < kQpWaves ? prc * B + qc : 0;  // the others: one request
        S.qp = (a.Qprev + tc * band::kTileRows * B)[off];
      }
    };
    auto store_row = [&](double* ad, const BandRow& R, int cmin) {
      // zero (82 16-B slots: lanes 0..63, then 0..17 again; lanes past 17 repeat slot 81),
      // then scatter entry 4 lane + k - shift; out-of-range entries select column kTrash
      constexpr int kTail = band::kAdLd / 2 - 64;
      d2v* ad2 = reinterpret_cast<d2v*>(ad);
      ad2[lane] = d2v{0.0, 0.0};
      ad2[64 + (lane < kTail ? lane : kTail - 1)] = d2v{0.0, 0.0};
      const int er = 4 * lane - R.shift;
      const int cc[4] = {R.c.x, R.c.y, R.c.z, R.c.w};
      const double vv[4] = {R.v0.x, R.v0.y, R.v1.x, R.v1.y};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int x = (unsigned)(er + k) < (unsigned)R.cnt ? cc[k] - cmin : band::kTrash;
        ad[perm8(x)] = vv[k];
      }
    };
    auto store_pair = [&](double* ad, const BandRow& R, int cnt0, int cmin) {
      constexpr int kTail = band::kAdLd / 2 - 64;
      d2v* ad2 = reinterpret_cast<d2v*>(ad);
      ad2[lane] = d2v{0.0, 0.0};
      ad2[64 + (lane < kTail ? lane : kTail - 1)] = d2v{0.0, 0.0};
      ad2[band::kAdLd / 2 + lane] = d2v{0.0, 0.0};
      ad2[band::kAdLd / 2 + 64 + (lane < kTail ? lane : kTail - 1)] = d2v{0.0, 0.0};
      const int er = 4 * lane - R.shift;
      const int cc[4] = {R.c.x, R.c.y, R.c.z, R.c.w};
      const double vv[4] = {R.v0.x, R.v0.y, R.v1.x, R.v1.y};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int x = (unsigned)(er + k) < (unsigned)R.cnt ? cc[k] - cmin : band::kTrash;
        const int row = er + k >= cnt0 ? band::kAdLd : 0;
        ad[row + perm8(x)] = vv[k];
      }
    };
    auto store_stage = [&](int64_t t, const BandStage& S, int buf) {
      if (t >= t1) return;
      double* ad = adb(buf) + 2 * p * band::kAdLd;
      if constexpr (PAIR) {
        store_pair(ad, S.r0, S.cnt0, S.cmin);
      } else {
        store_row(ad, S.r0, S.cmin);
        store_row(ad + band::kAdLd, S.r1, S.cmin);
      }
      if (p * (64 / B) < S.nnew) {  // wave-uniform: some new row among this wave's first
        const int l0 = qr < S.nnew ? qr : S.nnew - 1;
        *reinterpret_cast<double*>(smem + ring_addr(S.lo + l0, qc)) = S.q0;
      }
      if (p * (64 / B) + kQStep < S.nnew) {
        const int l1 = qr + kQStep < S.nnew ? qr + kQStep : S.nnew - 1;
        *reinterpret_cast<double*>(smem + ring_addr(S.lo + l1, qc)) = S.q1;
      }
      if constexpr (EPI) {
        if (p < kQpWaves) qpb(buf)[qp_off] = S.qp;
      }
      if (p == 0) {  // wave-uniform; every lane stores the same two words
        dsb(buf)[0] = S.cmin;
        dsb(buf)[1] = S.K;
      }
    };

    {
      BandStage S0, S1;
      S0.desc_next = load_desc(t0);
      load_stage(t0, S0);
      store_stage(t0, S0, 0);
      S1.desc_next = load_desc(t0 + 1);
      load_stage(t0 + 1, S1);
      store_stage(t0 + 1, S1, 1);
    }
    BandStage SA, SB, SC;
    SA.desc_next = load_desc(t0 + 2);
    SB.desc_next = load_desc(t0 + 3);
    SC.desc_next = load_desc(t0 + 4);
    load_stage(t0 + 2, SA);
    load_stage(t0 + 3, SB);
    load_stage(t0 + 4, SC);
    __syncthreads();
    // phase t (relative index i = t - t0): write tile t+2 into buffer (i+2) % 3, refill
    auto phase = [&](int64_t t, BandStage& S, int buf) {
      const unsigned long long s0 = stamp();
      store_stage(t + 2, S, buf);
      const unsigned long long sm = stamp();
      load_stage(t + 2 + kRegStages, S);
      const unsigned long long s1 = stamp();
      __syncthreads();
      const unsigned long long s2 = stamp();
      if constexpr (PROF) { pw += s1 - s0; pb += s2 - s1; px += sm - s0; }
    };
    for (int64_t t = t0; t < t1; t += band::kBufs) {
      phase(t, SA, 2);
      if (t + 1 < t1) phase(t + 1, SB, 0);
      if (t + 2 < t1) phase(t + 2, SC, 1);
    }
  } else {
    // =============================== consumers ===============================
    const int cg = wave % NCG, h = wave / NCG;
    const int q = lane >> 4;
    const int bcol = 4 * cg + (lane & 3);
    // epilogue operand: B_i^T[k][c] = B_i[c][k] for this wave's column group and k-steps
    double bt[EPI ? EKS : 1];
    if constexpr (EPI) {
#pragma unroll
      for (int e = 0; e < EKS; ++e) {
        const int k = 4 * (h * EKS + e) + (lane >> 4);
        bt[e] = -a.Bi[(4 * cg + (lane & 3)) * B + k];
      }
    }
    double pend = 0.0;  // KSPLIT > 1, h == 0: accumulator awaiting its partner's half
    double ai[AIG ? NCG : 1];
#pragma unroll
    for (int c = 0; c < (AIG ? NCG : 1); ++c) ai[c] = 0.0;
    auto store_u = [&](int64_t t, double acc) {  // U rows padded to a multiple of 16
      const int g = (lane >> 2) & 3;
      (a.U + t * band::kTileRows * B)[(4 * g + (lane >> 4)) * B + bcol] = acc;
      if constexpr (AIG) {
        const int64_t rl = t * band::kTileRows + 4 * g + (lane >> 4);
        const double um = rl < a.nrows ? acc : 0.0;  // rows past the end: no share
        const int grow = (int)(a.row0 + rl);
#pragma unroll
        for (int qc = 0; qc < NCG; ++qc) {
          const double qv = *reinterpret_cast<const double*>(smem + ring_addr(grow, 4 * qc + (lane & 3)));
          ai[qc] = mfma4b(qv, um, ai[qc]);
        }
      }
    };
    auto compute = [&](int64_t t, int buf) {
      if (a.ablate == 1) return;  // diagnostics: pipeline only
      const int cmin = __builtin_amdgcn_readfirstlane(dsb(buf)[0]);
      const int K = __builtin_amdgcn_readfirstlane(dsb(buf)[1]);
      const int ks = (K + 3) >> 2;
      int kb = 0, ke = ks;
      if constexpr (KSPLIT > 1) {
        const int half = ((ks + 2 * KSPLIT - 1) / (2 * KSPLIT)) * 2;  // even: pairs align
        kb = h * half;
        ke = kb + half < ks ? kb + half : ks;
      }
      // lane (row r, q): column 4 k' + q sits at perm8(4 k' + q) = 8 (k'/2) + 2q + (k'&1)
      const double* ad = adb(buf) + (lane & 15) * band::kAdLd + 2 * q;
      // ring byte address of (row cmin + 4k' + q, col bcol): +4 rows per k-step; the
      // swizzle bit (row parity) is the same for every k'
      unsigned rb = ring_addr(cmin + 4 * kb + q, bcol);
      constexpr unsigned kStep = 4 * L::kRowBytes;
      double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
      int kk = kb;
      for (; kk + 4 <= ke; kk += 4) {
        const d2v a01 = *reinterpret_cast<const d2v*>(ad + 4 * kk);
        const d2v a23 = *reinterpret_cast<const d2v*>(ad + 4 * kk + 8);
        const double b0 = *reinterpret_cast<const double*>(smem + rb);
        const double b1 = *reinterpret_cast<const double*>(smem + ((rb + kStep) & kRingMask));
        const double b2 = *reinterpret_cast<const double*>(smem + ((rb + 2 * kStep) & kRingMask));
        const double b3 = *reinterpret_cast<const double*>(smem + ((rb + 3 * kStep) & kRingMask));
        rb = (rb + 4 * kStep) & kRingMask;
        acc0 = mfma4b(a01.x, b0, acc0);
        acc1 = mfma4b(a01.y, b1, acc1);
        acc2 = mfma4b(a23.x, b2, acc2);
        acc3 = mfma4b(a23.y, b3, acc3);
      }
      if (kk + 2 <= ke) {
        const d2v a01 = *reinterpret_cast<const d2v*>(ad + 4 * kk);
        const double b0 = *reinterpret_cast<const double*>(smem + rb);
        const double b1 = *reinterpret_cast<const double*>(smem + ((rb + kStep) & kRingMask));
        rb = (rb + 2 * kStep) & kRingMask;
        acc0 = mfma4b(a01.x, b0, acc0);
        acc1 = mfma4b(a01.y, b1, acc1);
        kk += 2;
      }
      if (kk < ke) acc2 = mfma4b(ad[4 * kk], *reinterpret_cast<const double*>(smem + rb), acc2);
      if constexpr (EPI) {
        const double* qp = qpb(buf) + (lane & 15) * QPLD + 2 * q;
        if constexpr (EKS % 2 == 0) {
#pragma unroll
          for (int e = 0; e < EKS; e += 2) {
            const d2v qv = *reinterpret_cast<const d2v*>(qp + 8 * ((h * EKS + e) >> 1));
            if ((e >> 1) & 1) {
              acc2 = mfma4b(qv.x, bt[e], acc2);
              acc3 = mfma4b(qv.y, bt[e + 1], acc3);
            } else {
              acc0 = mfma4b(qv.x, bt[e], acc0);
              acc1 = mfma4b(qv.y, bt[e + 1], acc1);
            }
          }
        } else {
#pragma unroll
          for (int e = 0; e < EKS; ++e) acc3 = mfma4b(qp[perm8(4 * (h * EKS + e))], bt[e], acc3);
        }
      }
      const double acc = (acc0 + acc1) + (acc2 + acc3);
      if constexpr (KSPLIT == 1) {
        store_u(t, acc);
      } else if (h > 0) {
        xcb(t & 1)[((h - 1) * NCG + cg) * 64 + lane] = acc;
      } else {
        pend = acc;
      }
    };
    auto finalize = [&](int64_t t) {  // KSPLIT > 1: after the barrier that follows compute(t)
      if constexpr (KSPLIT > 1) {
        if (h != 0) return;
        double acc = pend;
#pragma unroll
        for (int s = 1; s < KSPLIT; ++s) acc += xcb(t & 1)[((s - 1) * NCG + cg) * 64 + lane];
        store_u(t, acc);
      }
    };
    __syncthreads();
    auto phase = [&](int64_t t, int buf) {
      const unsigned long long s0 = stamp();
      if (t > t0) finalize(t - 1);
      compute(t, buf);
      const unsigned long long s1 = stamp();
      __syncthreads();
      const unsigned long long s2 = stamp();
      if constexpr (PROF) { pw += s1 - s0; pb += s2 - s1; }
    };
    for (int64_t t = t0; t < t1; t += band::kBufs) {
      phase(t, 0);
      if (t + 1 < t1) phase(t + 1, 1);
      if (t + 2 < t1) phase(t + 2, 2);
    }
    finalize(t1 - 1);
    if constexpr (AIG) {
      if (KSPLIT == 1 || h == 0) {  // the waves that stored U own its column groups
        const int g = (lane >> 2) & 3;
        double* out = a.ai_slab + (int64_t)blockIdx.x * B * B;
#pragma unroll
        for (int qc = 0; qc < NCG; ++qc) {
          double v = ai[qc];
          v += __shfl_xor(v, 4, 64);
          v += __shfl_xor(v, 8, 64);
          if (g == 0) out[(4 * qc + (lane >> 4)) * B + bcol] = v;
        }
      }
    }
  }
  if constexpr (PROF) {
    if (lane == 0) {
      atomicAdd(a.prof + wave * 4 + 0, pw);
      atomicAdd(a.prof + wave * 4 + 1, pb);
      atomicAdd(a.prof + wave * 4 + 2, px);
      atomicAdd(a.prof + wave * 4 + 3, (unsigned long long)(t1 - t0));
    }
  }
}

template <int B, bool EPI, bool AIG, bool PAIR>
static void launch_band_t(const BandArgs& a0, int grid, hipStream_t s) {
  static bool attr = false;
  static const bool prof = [] {
    const char* e = getenv("RBL_SPMM_PROF");
    return e && atoi(e) != 0;
  }();
  if (!attr) {
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_spmm_band<B, EPI, false, AIG, PAIR>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, BandLayout<B>::kLds);
    (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&k_spmm_band<B, EPI, true, AIG, PAIR>),
                              hipFuncAttributeMaxDynamicSharedMemorySize, BandLayout<B>::kLds);
    attr = true;
  }
  if (!prof) {
    hipLaunchKernelGGL((k_spmm_band<B, EPI, false, AIG, PAIR>), dim3(grid), dim3(band::kThreads),
                       BandLayout<B>::kLds, s, a0);
    return;
  }
  // diagnostics: work / barrier cycles per wave and tile, printed to stderr
  BandArgs a = a0;
  static unsigned long long* d = nullptr;
  if (!d) (void)hipMalloc(&d, 64 * sizeof(unsigned long long));
  (void)hipMemsetAsync(d, 0, 64 * sizeof(unsigned long long), s);
  a.prof = d;
  hipLaunchKernelGGL((k_spmm_band<B, EPI, true, AIG, PAIR>), dim3(grid), dim3(band::kThreads),
                     BandLayout<B>::kLds, s, a);
  unsigned long long hbuf[64];
  (void)hipMemcpyAsync(hbuf, d, sizeof(hbuf), hipMemcpyDeviceToHost, s);
  (void)hipStreamSynchronize(s);
  for (int w : {0, 3, 7, 8, 11, 15}) {
    const double tiles = (double)hbuf[w * 4 + 3];
    fprintf(stderr, "band prof b=%d epi=%d wave %2d (%s): per tile work %.0f (store %.0f) barrier %.0f cycles\n",
            B, (int)EPI, w, w < band::kConsumers ? "consumer" : "producer", hbuf[w * 4] / tiles,
            hbuf[w * 4 + 2] / tiles, hbuf[w * 4 + 1] / tiles);
  }
}

bool spmm_band(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
               const double* Qprev, const double* Bi, hipStream_t s, double* ai_slab,
               int* ai_parts) {
  if (A.ntiles <= 0 || !((b == 16 && A.band_ok16) || (b == 32 && A.band_ok32))) return false;
  BandArgs a;
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
  static const int ablate = [] {
    const char* e = getenv("RBL_SPMM_ABLATE");
    return e ? atoi(e) : 0;
  }();
  a.ablate = ablate;
  a.prof = nullptr;
  a.row0 = A.row0;
  const int grid = (int)((A.ntiles + A.tiles_per_wg - 1) / A.tiles_per_wg);
  const bool epi = Qprev != nullptr;
  const bool aig = ai_slab != nullptr && A.band_gram;
  a.ai_slab = aig ? ai_slab : nullptr;
  if (ai_parts) *ai_parts = aig ? grid : 0;
  // every combination is its own kernel (template flags): pick by (b, epilogue, A_i, pair)
  const int key = (b == 32 ? 8 : 0) | (epi ? 4 : 0) | (aig ? 2 : 0) | (A.band_pair ? 1 : 0);
  switch (key) {
#define RBL_BAND_CASE(K, BB, E, G, P) \
    case K: launch_band_t<BB, E, G, P>(a, grid, s); break;
    RBL_BAND_CASE(0, 16, false, false, false) RBL_BAND_CASE(1, 16, false, false, true)
    RBL_BAND_CASE(2, 16, false, true, false)  RBL_BAND_CASE(3, 16, false, true, true)
    RBL_BAND_CASE(4, 16, true, false, false)  RBL_BAND_CASE(5, 16, true, false, true)
    RBL_BAND_CASE(6, 16, true, true, false)   RBL_BAND_CASE(7, 16, true, true, true)
    RBL_BAND_CASE(8, 32, false, false, false) RBL_BAND_CASE(9, 32, false, false, true)
    RBL_BAND_CASE(10, 32, false, true, false) RBL_BAND_CASE(11, 32, false, true, true)
    RBL_BAND_CASE(12, 32, true, false, false) RBL_BAND_CASE(13, 32, true, false, true)
    RBL_BAND_CASE(14, 32, true, true, false)  RBL_BAND_CASE(15, 32, true, true, true)
#undef RBL_BAND_CASE
  }
  return true;
}

}  // namespace rbl
