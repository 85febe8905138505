// spmm_band.hip — persistent CSR SpMM for banded sparsity with the band tile densified in
// LDS and multiplied on fp64 MFMA (gfx950).
//
// U = A * Q_i (+ fused 3-term epilogue U -= Q_{i-1} B_i^T) — RBL_gpu.jl:176-177.
// HBM traffic: the CSR values (8 B per nonzero) and each nonzero's 16-bit band position
// (2 B, precomputed once per matrix from the CSR columns: band_positions), row pointers, plus
// Q_i, Q_{i-1} and U once.
//
// Why densify: a row-per-nonzero kernel (spmm_window.hip) reads one b*8-byte Q row from LDS
// per nonzero; at n=1e7, nnz=1e9, b=32 that is 256 GB of LDS reads — as long as the whole
// HBM stream.  Here each 16-row tile's band is scattered into a dense LDS tile and
// multiplied with the Q ring rows by v_mfma_f64_4x4x4f64: every Q ring row is read once per
// tile (not once per nonzero).
//
// The budget that matters (tools/coexec_probe.hip): on gfx950 the fp64 4x4x4 MFMA does not
// co-execute with VALU instructions of any kind, so a SIMD's time per tile is its MFMA cycles
// PLUS every VALU cycle of its four waves.  The layout is chosen to spend almost no VALU:
//   * the band of tile t starts at c16 = cmin(t) & ~15, so the consumers walk it in groups of
//     16 columns (4 k-steps) whose 16 ring rows never straddle the ring's wrap: one VALU add
//     per group for the ring address, immediate offsets for everything else;
//   * each nonzero carries its precomputed byte offset in the dense tile (row, perm8 column),
//     so the producers' scatter is a bounds select per entry (no column arithmetic);
//   * loads use SGPR bases and lane-constant offsets (CSR over-reads land in kCsrPad).
//
// Workgroup: 1024 threads (16 waves), one per CU, persistent over a contiguous tile range,
// split by role, one barrier per tile:
//   * waves 8..15 produce: in phase t they move the register-staged data of tile t+2 into
//     LDS (zero + scatter two dense rows per wave, the tile's new Q ring rows, its Q_{i-1}
//     rows) and issue the global loads of tile t+2+kRegStages;
//   * waves 0..7 consume: in phase t they multiply tile t — wave c owns column group
//     cg = c % (b/4) (and band half h = c / (b/4) at b=16), four accumulators, the operands
//     of group j+2 read while group j multiplies — then the fused 3-term epilogue, the store
//     of U and (AIG) the partials of A_i = Q_i^T U.
//   Dense tiles, Q_{i-1} tiles and tile descriptors are triple-buffered (compute t, staged
//   t+1, being written t+2).
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
constexpr int kGroupK = 16;           // band columns per consumer group (4 k-steps)
constexpr int kMaxK = kBandMaxK;      // 176: band [c16, cmax] incl. the alignment shift
// dense tile rows: column x stored at perm8(x) so a lane's k-steps u, u+1 (columns x, x+4)
// come in one ds_read_b128; kAdLd = 4 mod 32 puts the 16 rows of each ds_read_b128 lane group
// on distinct 16-B bank slots (slot = 2 row + q mod 16).  Column kTrash is the scatter's
// discard slot (never multiplied: groups cover columns < kMaxK).
constexpr int kAdLd = kBandLd;
constexpr int kTrash = kMaxK;
constexpr int kRing = kBandRing;      // ring rows (power of two: slot = row & (kRing - 1))
constexpr int kBufs = 3;
static_assert(perm8(kTrash) == kTrash && kTrash < kAdLd && kAdLd % 32 == 4, "tile layout");
static_assert(kMaxK % kGroupK == 0 && kTileRows * kAdLd * 8 < 65536, "16-bit positions");
static_assert((kConsumers + kProducers) * 64 == kThreads && 2 * kProducers == kTileRows,
              "roles: 8 consumer waves, 8 producer waves of two tile rows");
}  // namespace band
// CSR entries: a producer lane holds entries 4l..4l+3 counted from the row start rounded down
// to a multiple of 4 (8-B aligned position / 32-B aligned value loads): a row (or row pair)
// of up to 253 nonzeros in one uint2 + two double2 loads per lane.

__device__ __forceinline__ double mfma4b(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}

struct BandArgs {
  int64_t nrows;
  int64_t ntiles;
  int64_t tiles_per_wg;
  const int64_t* rowptr;
  const uint16_t* pos;   // band positions, padded by kCsrPad entries
  const double* val;     // padded by kCsrPad entries
  const int64_t* tinfo;  // per tile: e0, nnz, lo, hi, cmin, cmax, 0, 0
  const double* Q;       // rows [col_off, ...) of the halo-extended Q
  int64_t col_off;
  double* U;             // padded to a multiple of 16 rows
  const double* Qprev;
  const double* Bi;
  double* ai_slab;           // AIG: per-workgroup partials of A_i = Q[own rows]^T U (b x b)
  int64_t row0;              // global index of local row 0 (ring rows are global)
  int ablate;                // diagnostics only (RBL_SPMM_ABLATE: 1 skip compute, 2 skip the
                             // dense-tile zero/scatter, 3 both)
  unsigned long long* prof;  // diagnostics only (PROF instantiation)
};

template <int B>
struct BandLayout {
  static constexpr int NCG = B / 4;                   // column groups of 4
  static constexpr int KSPLIT = band::kConsumers / NCG;  // consumer waves per column group
  // ring row = B doubles, no padding: at b=32 the two rows a 32-lane half reads in one
  // ds_read_b64 (q = 0/1 or 2/3) would share banks, so column c of ring row r is stored at
  // c ^ ((r & 1) << 2) (4 columns = 8 banks apart); at b=16 rows r, r+1 are 32 banks apart.
  // The consumers' rows c16 + 16j + 4u + q have parity q & 1: a lane-constant column.
  static constexpr int kSwz = B == 32 ? 4 : 0;
  static constexpr int kRowBytes = B * 8;
  static constexpr int kRingBytes = band::kRing * kRowBytes;   // 64 KiB / 32 KiB
  static constexpr int kQRows = 512 / B;       // ring rows one producer pass stores
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
  int cnt;    // entries of the row (pair)
  int shift;  // row start - 4-aligned start (0..3)
  uint2 pk;   // four 16-bit band positions
  d2v v0, v1;
};

// PAIR staging: the two rows of a producer wave are contiguous in CSR, so one set of lane
// loads (64 lanes x 4 entries) covers both when their nonzeros + alignment shift fit 256
// (checked on the host: CsrDev::band_pair); r0 then holds the pair and r1 is unused.  The
// positions carry the row, so the pair scatters like one row.
struct BandStage {
  int64_t desc_next;  // lane l <= 16: rowptr[16T'+l]; 17..20: lo, hi, cmin, cmax of the next tile
  int nnew, lo, c16, ng;  // of the tile the registers below hold (wave-uniform)
  BandRow r0, r1;
  double q0, q1;      // new ring rows, up to two elements per producer thread
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
  constexpr int RB = L::kRowBytes;
  constexpr int EKS = (B / 4) / KSPLIT;  // epilogue k-steps per consumer wave
  constexpr int kRegStages = 3;          // register sets of prefetched tile data
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
    return ((unsigned)(row & (band::kRing - 1)) * RB) + (unsigned)((col ^ ((row & 1) ? L::kSwz : 0)) * 8);
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

  // ---- prologue: zero ring (finite everywhere: groups read rows outside the band, whose
  // zero A columns meet them), then the first tile's band rows, by every thread ----
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
    constexpr int kQRows = L::kQRows;
    const int qr = ptid / B, qc = ptid % B;
    const int qp_off = qr * QPLD + perm8(qc);   // qr < 16 for the threads that store Q_{i-1}
    constexpr int kQpWaves = band::kTileRows * B / 64;  // producer waves storing Q_{i-1}
    // zero fill of rows 2p, 2p+1: kAdLd 16-B slots, lanes 0..63 three times, then 192..195
    const unsigned zrow = (unsigned)(2 * p * band::kAdLd * 8);
    const unsigned z0 = zrow + 16u * lane, z3 = zrow + 16u * (192 + (lane < 4 ? lane : 3));
    static_assert(band::kAdLd == 196, "zero fill covers 196 slots");
    constexpr unsigned kTrashByte = band::kTrash * 8;

    auto load_row = [&](int64_t rs, int cnt, BandRow& R) {
      R.cnt = cnt;
      R.shift = (int)(rs & 3);
      const int64_t ra = rs - R.shift;  // lanes past the row read on: the entries go to trash
      R.pk = reinterpret_cast<const uint2*>(a.pos + ra)[lane];
      R.v0 = reinterpret_cast<const d2v*>(a.val + ra)[2 * lane];
      R.v1 = reinterpret_cast<const d2v*>(a.val + ra)[2 * lane + 1];
    };
    // take the descriptor loaded kRegStages phases ago, issue tile t's loads and the
    // descriptor load of tile t + kRegStages
    auto load_stage = [&](int64_t t, BandStage& S) {
      const int rs_lo = lane32(S.desc_next, 2 * p);
      const int rs_hi = __builtin_amdgcn_readlane((int)(S.desc_next >> 32), 2 * p);
      const int64_t rs = ((int64_t)rs_hi << 32) | (unsigned)rs_lo;
      const int m_lo = lane32(S.desc_next, 2 * p + 1), e_lo = lane32(S.desc_next, 2 * p + 2);
      const int lo = lane32(S.desc_next, 17), hi = lane32(S.desc_next, 18);
      const int cmin = lane32(S.desc_next, 19), cmax = lane32(S.desc_next, 20);
      S.c16 = cmin & ~15;
      S.ng = (cmax - S.c16 + band::kGroupK) / band::kGroupK;
      S.lo = lo;
      S.nnew = hi - lo;
      S.desc_next = load_desc(t + kRegStages);
      if constexpr (PAIR) {
        load_row(rs, e_lo - rs_lo, S.r0);  // both rows: one load set
      } else {
        load_row(rs, m_lo - rs_lo, S.r0);
        load_row(rs + (m_lo - rs_lo), e_lo - m_lo, S.r1);
      }
      // new ring rows lo + qr (+ kQRows), clamped to the last new row (threads past it
      // re-read and later re-store that row's data); no new row: any band row
      const int rlast = S.nnew > 0 ? hi - 1 : cmin;
      const double* qb = a.Q - a.col_off * B + qc;
      const int ra0 = lo + qr < rlast ? lo + qr : rlast;
      S.q0 = qb[(int64_t)ra0 * B];
      if (S.nnew > kQRows) {  // wave-uniform, rare (C4a: 16 new rows per tile)
        const int ra1 = lo + kQRows + qr < rlast ? lo + kQRows + qr : rlast;
        S.q1 = qb[(int64_t)ra1 * B];
      }
      if constexpr (EPI) {
        const int64_t tc = t < t1 ? t : t1 - 1;
        const int64_t last = a.nrows - 1 - tc * band::kTileRows;  // >= 0
        const int prc = qr < last ? qr : (int)last;
        const int off = p < kQpWaves ? prc * B + qc : 0;  // the others: one request
        S.qp = (a.Qprev + tc * band::kTileRows * B)[off];
      }
    };
    // scatter entry k of each lane to its precomputed position, or to the trash slot when it
    // lies outside the row (pair): one compare + select per entry
    auto store_row = [&](unsigned char* ab, const BandRow& R) {
      const int er = 4 * lane - R.shift;
      const unsigned pk[4] = {R.pk.x & 0xffffu, R.pk.x >> 16, R.pk.y & 0xffffu, R.pk.y >> 16};
      const double vv[4] = {R.v0.x, R.v0.y, R.v1.x, R.v1.y};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const unsigned x = (unsigned)(er + k) < (unsigned)R.cnt ? pk[k] : kTrashByte;
        *reinterpret_cast<double*>(ab + x) = vv[k];
      }
    };
    auto store_stage = [&](int64_t t, const BandStage& S, int buf) {
      if (t >= t1) return;
      unsigned char* ab = smem + L::kAdOff + buf * L::kAdBytes;
      if (!(a.ablate & 2)) {  // (diagnostics: RBL_SPMM_ABLATE bit 1 skips the dense tile,
        if (!(a.ablate & 4)) {  // bit 2 its zero fill, bit 3 its scatter)
          const d2v z = {0.0, 0.0};
          *reinterpret_cast<d2v*>(ab + z0) = z;
          *reinterpret_cast<d2v*>(ab + z0 + 1024) = z;
          *reinterpret_cast<d2v*>(ab + z0 + 2048) = z;
          *reinterpret_cast<d2v*>(ab + z3) = z;
        }
        if (!(a.ablate & 8)) {
          store_row(ab, S.r0);
          if constexpr (!PAIR) store_row(ab, S.r1);
        }
      }
      {
        const int rlast = S.nnew > 0 ? S.lo + S.nnew - 1 : S.c16;  // as in load_stage
        const int r = S.lo + qr < rlast ? S.lo + qr : rlast;
        if (S.nnew > 0) *reinterpret_cast<double*>(smem + ring_addr(r, qc)) = S.q0;
        if (S.nnew > kQRows) {
          const int r1 = S.lo + kQRows + qr < rlast ? S.lo + kQRows + qr : rlast;
          *reinterpret_cast<double*>(smem + ring_addr(r1, qc)) = S.q1;
        }
      }
      if constexpr (EPI) {
        if (p < kQpWaves) qpb(buf)[qp_off] = S.qp;
      }
      if (p == 0) {  // wave-uniform; every lane stores the same two words
        dsb(buf)[0] = S.c16;
        dsb(buf)[1] = S.ng;
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
    // lane part of the ring byte address of (row c16 + 16j + 4u + q, col bcol): row parity q & 1
    const unsigned bl = (unsigned)(q * RB + ((bcol ^ ((q & 1) ? L::kSwz : 0)) * 8));
    // epilogue operand: B_i^T[k][c] = B_i[c][k] for this wave's column group and k-steps
    double bt[EPI ? EKS : 1];
    if constexpr (EPI) {
#pragma unroll
      for (int e = 0; e < EKS; ++e) {
        const int k = 4 * (h * EKS + e) + (lane >> 4);
        bt[e] = -a.Bi[(4 * cg + (lane & 3)) * B + k];
      }
    }
    // AIG ring reads of the tile's own rows r = row0 + 16t + 4g + q: the swizzle parity
    // (row0 + q) & 1 is lane-constant, so column 4qc + (lane&3) sits at 32 (qc ^ s) + 8 (lane&3)
    // = 32 qc + (qc even ? ao_e : ao_o)
    const int g4 = 4 * ((lane >> 2) & 3) + q;
    const int as = L::kSwz && ((a.row0 + q) & 1) ? 1 : 0;
    const unsigned ao_e = 8u * (lane & 3) + (as ? 32u : 0u), ao_o = 8u * (lane & 3) - (as ? 32u : 0u);
    double pend = 0.0;  // KSPLIT > 1, h == 0: accumulator awaiting its partner's half
    double ai[AIG ? NCG : 1];
#pragma unroll
    for (int c = 0; c < (AIG ? NCG : 1); ++c) ai[c] = 0.0;
    auto store_u = [&](int64_t t, double acc) {  // U rows padded to a multiple of 16
      (a.U + t * band::kTileRows * B)[g4 * B + bcol] = acc;
      if constexpr (AIG) {
        const int64_t rl = t * band::kTileRows + g4;
        const double um = rl < a.nrows ? acc : 0.0;  // rows past the end: no share
        const unsigned rb = (unsigned)((a.row0 + t * band::kTileRows + g4) & (band::kRing - 1)) * RB;
        const unsigned be = rb + ao_e, bo = rb + ao_o;  // 32-bit sums: bo + 32 qc >= rb (qc odd)
#pragma unroll
        for (int qc = 0; qc < NCG; ++qc) {
          const double qv = *reinterpret_cast<const double*>(smem + ((qc & 1 ? bo : be) + 32u * qc));
          ai[qc] = mfma4b(qv, um, ai[qc]);
        }
      }
    };
    auto compute = [&](int64_t t, int buf) {
      if (a.ablate & 1) return;  // diagnostics: pipeline only
      const int c16 = __builtin_amdgcn_readfirstlane(dsb(buf)[0]);
      const int ng = __builtin_amdgcn_readfirstlane(dsb(buf)[1]);
      int gb = 0, ge = ng;
      if constexpr (KSPLIT > 1) {
        const int half = (ng + 1) >> 1;
        gb = h ? half : 0;
        ge = h ? ng : half;
      }
      double acc0 = 0.0, acc1 = 0.0, acc2 = 0.0, acc3 = 0.0;
      // lane (row r, q): column 16j + 4u + q sits at perm8 = 16j + 8(u>>1) + 2q + (u&1)
      const double* ad = adb(buf) + (lane & 15) * band::kAdLd + 2 * q + band::kGroupK * gb;
      int j = 0;
      const int n = ge - gb;
      struct Grp {
        d2v x01, x23;
        double b[4];
      };
      // group j's operands: A two ds_read_b128, B four ds_read_b64 at one base (16 ring rows
      // never straddle the wrap: c16 is 16-aligned) — one VALU add per group
      auto ld = [&](int jj) -> Grp {
        Grp G;
        G.x01 = *reinterpret_cast<const d2v*>(ad + band::kGroupK * jj);
        G.x23 = *reinterpret_cast<const d2v*>(ad + band::kGroupK * jj + 8);
        const unsigned sb = ((unsigned)(c16 + band::kGroupK * (gb + jj)) & (band::kRing - 1)) * RB;
        const unsigned char* bp = smem + sb + bl;
#pragma unroll
        for (int u = 0; u < 4; ++u) G.b[u] = *reinterpret_cast<const double*>(bp + u * 4 * RB);
        return G;
      };
      auto pin = [](Grp& G) {
        asm volatile("" : "+v"(G.x01), "+v"(G.x23), "+v"(G.b[0]), "+v"(G.b[1]), "+v"(G.b[2]), "+v"(G.b[3]));
      };
      // software-pipelined two groups ahead: group j+2's reads issue before group j's MFMAs;
      // group j+1's (read one step ago) are pinned after them — without the pin LLVM sinks
      // the read-ahead past the loop exit and every group waits on its own LDS latency.
      // Read-ahead past the band is harmless: in-bounds LDS, never multiplied.
      auto step = [&](const Grp& cur, Grp& mid, Grp& nx) -> bool {
        nx = ld(j + 2);
        acc0 = mfma4b(cur.x01.x, cur.b[0], acc0);
        acc1 = mfma4b(cur.x01.y, cur.b[1], acc1);
        acc2 = mfma4b(cur.x23.x, cur.b[2], acc2);
        acc3 = mfma4b(cur.x23.y, cur.b[3], acc3);
        pin(mid);
        return ++j < n;
      };
      if (n > 0) {
        Grp c0 = ld(0), c1 = ld(1), c2;
        while (step(c0, c1, c2) && step(c1, c2, c0) && step(c2, c0, c1)) {
        }
      }
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
  ensure_lds_attr(reinterpret_cast<const void*>(&k_spmm_band<B, EPI, false, AIG, PAIR>), BandLayout<B>::kLds);
#ifndef RBL_VARIANTS
  hipLaunchKernelGGL((k_spmm_band<B, EPI, false, AIG, PAIR>), dim3(grid), dim3(band::kThreads),
                     BandLayout<B>::kLds, s, a0);
#else
  static const bool prof = [] {
    const char* e = getenv("RBL_SPMM_PROF");
    return e && atoi(e) != 0;
  }();
  ensure_lds_attr(reinterpret_cast<const void*>(&k_spmm_band<B, EPI, true, AIG, PAIR>), BandLayout<B>::kLds);
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
#endif
}

bool spmm_band(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
               const double* Qprev, const double* Bi, hipStream_t s, double* ai_slab,
               int* ai_parts) {
  if (A.ntiles <= 0 || !A.band_pos || !((b == 16 && A.band_ok16) || (b == 32 && A.band_ok32)))
    return false;
  BandArgs a;
  a.nrows = A.nrows;
  a.ntiles = A.ntiles;
  a.tiles_per_wg = A.tiles_per_wg;
  a.rowptr = A.rowptr;
  a.pos = A.band_pos;
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

// ---- band positions (once per matrix) --------------------------------------------------
// pos[e] = ((r % 16) * kAdLd + perm8(col[e] - c16(r / 16))) * 8 for every nonzero e of row r.
__global__ void k_band_pos(int64_t nrows, const int64_t* __restrict__ rowptr,
                           const int32_t* __restrict__ col, const int64_t* __restrict__ tinfo,
                           uint16_t* __restrict__ pos) {
  // one wave per row, lanes over the row's entries
  const int64_t r = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (r >= nrows) return;
  const int64_t t = r / band::kTileRows;
  const int c16 = (int)(tinfo[8 * t + 4] & ~15ll);
  const int rr = (int)(r % band::kTileRows);
  for (int64_t e = rowptr[r] + lane; e < rowptr[r + 1]; e += 64)
    pos[e] = (uint16_t)((rr * band::kAdLd + perm8(col[e] - c16)) * 8);
}

void band_positions(const CsrDev& A, uint16_t* pos, hipStream_t s) {
  if (A.nrows <= 0) return;
  const int64_t threads = A.nrows * 64;
  hipLaunchKernelGGL(k_band_pos, dim3((unsigned)((threads + 255) / 256)), dim3(256), 0, s, A.nrows,
                     A.rowptr, A.col, A.tile_info, pos);
}

}  // namespace rbl
