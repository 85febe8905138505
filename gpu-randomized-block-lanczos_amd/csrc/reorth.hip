// reorth.hip — fp64 tall-skinny GEMMs on v_mfma_f64_4x4x4f64 (gfx950).
//
// Measured on MI355X (tools/mfma_probe.hip): the 4-block 4x4x4 fp64 MFMA sustains ~71 TF/s,
// the 16x16x4 shape ~46 TF/s, so the compute-heavy GEMMs of the block step use 4x4x4:
//   * k_gram44:  C = W^T X  with W the Krylov basis (m panels) and X = [Q_i, Q_{i-1}] —
//                the partial-reorth coefficients of RBL_gpu.jl:33,39 (part_reorth_gpu_async!)
//                batched over every j (block CGS, one launch instead of 2(i-2) gemms);
//   * k_tsmm44:  Y = beta Y + alpha X C  with X a run of panels — the partial-reorth update
//                (RBL_gpu.jl:34,40), the 3-term / local-reorth updates, CholQR apply and the
//                Ritz projection V = [Q_1..Q_m] S (RBL_gpu.jl:121, RBL.jl:68).
//
// v_mfma_f64_4x4x4f64 lane layout (tools/mfma_layout_probe.hip), block g = (lane>>2)&3:
//   A[i = lane&3][k = lane>>4], B[k = lane>>4][j = lane&3], D[i = lane>>4][j = lane&3].
// With the 4 blocks on 4 consecutive row-quads, the A operand of a wave is
//   M[r0 + (lane&15)][k0 + (lane>>4)]  (Gram: W^T -> W[r0+(lane>>4)][a0+(lane&15)]),
// i.e. 16 consecutive doubles per k — coalesced 128-B segments.
#include <algorithm>
#include <cstdlib>

#include "kernels.hpp"

namespace rbl {

__device__ __forceinline__ double mfma4(double a, double b, double c) {
  return __builtin_amdgcn_mfma_f64_4x4x4f64(a, b, c, 0, 0, 0);
}
// The Krylov basis W is read once per launch (up to 92 GB at C4a: no L2 / Infinity Cache
// reuse); non-temporal loads measured no faster here (596 vs 600 ms per run), so off
// RBL_REORTH_ABL (diagnostics only, wrong results): bit 0 drops the next chunk's basis loads
// (the MFMAs reuse the current operands), bit 1 the per-chunk barrier, bit 2 the LDS staging
// store of the next chunk — in k_gram44 and k_tsmm44f
#ifndef RBL_REORTH_ABL
#define RBL_REORTH_ABL 0
#endif
#ifndef RBL_REORTH_NT
#define RBL_REORTH_NT 0
#endif
template <typename T>
__device__ __forceinline__ T ldw(const T* p) {
  if constexpr (RBL_REORTH_NT) return __builtin_nontemporal_load(p);
  return *p;
}

// ----------------------------------------------------------------------------------------
// Gram C = W^T X: one Krylov panel per wave, 4 waves per workgroup (three workgroups per CU:
// while one waits at its per-chunk barrier the others keep the MFMA pipe busy), X rows
// staged in LDS in 16-row chunks shared by the 4 waves, A operands prefetched one chunk ahead.
// A last panel group with r < 4 panels splits the X columns over 4 / r waves per panel, so
// the even panel counts partial reorth produces leave no wave idle (tools/gram_probe.hip:
// idle waves cost ~25% at 18 panels with 8-wave groups).
// ----------------------------------------------------------------------------------------
constexpr int kG44Waves = 4;
#ifndef RBL_G44_ROWS
#define RBL_G44_ROWS 16
#endif
// 3 waves per SIMD (160 VGPRs); forcing 4 (128 VGPRs, 15 spilled) measured 9 % slower on the
// probe (287 vs 264 ms, profiles/r03_gram_wpe4_ab.log)
#ifndef RBL_G44_WPE
#define RBL_G44_WPE 3
#endif
#ifndef RBL_G44_PF
#define RBL_G44_PF 2
#endif
#ifndef RBL_G44_W16
#define RBL_G44_W16 1
#endif
// b = 16 (panel pairs): basis operands this many chunks ahead (2 or 3).  A 16-row chunk is half
// the MFMAs of a b = 32 chunk, so the same distance covers half the time
#ifndef RBL_G44_PF16
#define RBL_G44_PF16 RBL_G44_PF
#endif
// interleaved row splits (see k_gram44): b = 32 / b = 16
#ifndef RBL_G44_INTER
#define RBL_G44_INTER 0
#endif
#ifndef RBL_G44_INTER16
#define RBL_G44_INTER16 RBL_G44_INTER
#endif
#ifndef RBL_G44_WPE16
// b = 16 (panel pairs, HBM-bound at ~5 TB/s): 4 waves per SIMD (106 VGPRs) measured neutral on
// the probe and 0.5-0.8 % slower on the C2 / C3 lines (profiles/r03_gram16_wpe4_ab.log); the
// update spills at 4 (RBL_T44_WPE16), so both stay at 3
#define RBL_G44_WPE16 RBL_G44_WPE
#endif
#ifndef RBL_T44_WPE16
#define RBL_T44_WPE16 3
#endif
#ifndef RBL_G44_DUO_WPE
#define RBL_G44_DUO_WPE 1
#endif
#ifndef RBL_G44_GLDS
#define RBL_G44_GLDS 1
#endif
// b = 16: the X chunk by LDS-DMA as well?  While a global_load_lds is in flight hipcc (ROCm 7.2)
// closes every __syncthreads() with vmcnt(0), which also drains the basis prefetch issued for two
// chunks ahead (cdna_hip_programming.md, 'Pipelining across barriers'): the prefetch then covers
// one chunk.  Register staging keeps it (the barrier waits vmcnt(8): the X loads only)
#ifndef RBL_G44_GLDS16
#define RBL_G44_GLDS16 RBL_G44_GLDS
#endif
constexpr int kG44Rows = RBL_G44_ROWS;
typedef __attribute__((address_space(3))) void* lds_vptr;
typedef __attribute__((address_space(1))) void* glb_vptr;
constexpr int kLine = 136;  // doubles per LDS-DMA line: 1 KiB + 64 B pad

// GL (k_gram44): the X chunk (16 rows x KC, KC = 32 or 64) is staged by LDS-DMA
// (global_load_lds_dwordx4) into 1-KiB lines padded to 1088 B, row R at line
// (R & 3) + 4 ((R >> 2) / RPL), slot (R >> 2) % RPL: the rows 4ks + q (q = 0..3) one
// ds_read_b128 touches sit in 4 lines (conflict-free, lane offset q * 1088 + 16 (lane & 3)).
// Columns in natural order: lane (lane & 3) reads columns 8cp + 2(lane & 3) + {0, 1} (the
// register path stores perm8 order), which changes only the accumulator -> column map.  The
// rows of a shifted last chunk below rc0 are zeroed in LDS after the DMA lands.
template <int KC>
struct G44Lines {
  static constexpr int RPL = 1024 / (8 * KC);
  static constexpr int NL = kG44Rows * KC * 8 / 1024;  // lines per chunk
  __host__ __device__ static constexpr int off(int R) {
    return ((R & 3) + 4 * ((R >> 2) / RPL)) * kLine + ((R >> 2) % RPL) * KC;
  }
  __host__ __device__ static constexpr int row(int L, int s) { return 4 * (s + RPL * (L >> 2)) + (L & 3); }
};

// PAIR (B = 16): a wave's "panel" j is the pair of basis panels 2j, 2j+1 (32 columns, as one
// B = 32 panel: the same registers and MFMAs per chunk), so b = 16 runs the b = 32 tile shape
// DUO (B = 32, even panel count; RBL_G44_DUO=1, off by default): a wave's "panel" j is the pair
// of basis panels 2j, 2j+1 (64 columns, four column groups in two 16-B loads per row quad):
// twice the MFMAs per X operand read from LDS and half the panel groups.  Bit-identical, but
// measured slower (profiles/r03_gram_duo_ab.log): 289 ms summed over the probe at one wave per
// SIMD, 299 ms at two (19 VGPRs spilled), against 262 ms for one panel per wave at three waves
// per SIMD; C4a 45.4 vs 47.2 block-iters/s.  The extra waves hide the per-chunk barrier.
template <int B, int NX, int NPH, bool PAIR = false, bool GL = false, bool DUO = false>
__device__ __forceinline__ void gram44_body(int64_t r_begin, int64_t r_end, int64_t cs, int64_t s, int pg,
                                            int r, const PanelRun& W, const Panels& X,
                                            double* slab, double* xs_base) {
  constexpr int KC = NX * B;
  static_assert(!DUO || (B == 32 && !PAIR), "DUO: b = 32 panel pairs");
  constexpr int WB = PAIR || DUO ? 2 * B : B;  // basis columns per wave
  constexpr int AG = WB / 16;
  constexpr int CG = KC / 4;
  constexpr int CGP = CG / NPH;  // column groups of this wave (even: read in pairs)
  constexpr int LD = KC + 8;     // rows of a ds_read_b128 lane group differ by one: disjoint banks
  constexpr int EPT = kG44Rows * KC / (kG44Waves * 64);
  constexpr int KS = kG44Rows / 4;
  static_assert(CGP >= 2 && CGP % 2 == 0, "column split");
  using GLn = G44Lines<KC>;
  static_assert(!GL || ((KC == 32 || KC == 64) && kG44Rows == 16 && GLn::NL % kG44Waves == 0), "GL shape");
  constexpr int XB = GL ? GLn::NL * kLine : kG44Rows * LD;  // doubles per X buffer
  double(*xs)[XB] = reinterpret_cast<double(*)[XB]>(xs_base);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4;
  const int j = pg * kG44Waves + wave % r;  // panel
  const int ph = wave / r;                  // column phase
  const bool active = ph < NPH;
  const int cp0 = ph < NPH ? ph * (CGP / 2) : 0;

  double acc[AG][CGP];
#pragma unroll
  for (int ag = 0; ag < AG; ++ag)
#pragma unroll
    for (int cg = 0; cg < CGP; ++cg) acc[ag][cg] = 0.0;

  // Chunk c covers rows [rc0, rc0 + 16), rc0 = r_begin + 16c; a partial last chunk is shifted
  // back to end at r_end (rcl = min(rc0, r_end - 16), wave-uniform; nrows >= 16 on this path)
  // and its rows below rc0 — already counted — are zeroed on the X side, like rows past
  // r_end of the prefetch beyond the last chunk.  So every load is a wave-uniform row base
  // plus a lane constant: no per-lane clamps in the loop (fp64 MFMA does not co-execute
  // with VALU on gfx950).
  const int xe0 = tid * EPT;
  const int xrow = xe0 / KC, xcol = xe0 % KC;
  const double* xsl = X.ptr[xcol / B] + (xcol % B) + (int64_t)xrow * B;
  // column group ag of the wave's panel (PAIR: ag = the pair member).  W16 (b = 32): lane
  // column 2 (lane & 15) + ag, both ag in one 16-B load (W16 = 0: columns (lane & 15) + 16 ag,
  // two 8-B loads); the MFMAs see the same operands per output, only C's row order differs
  constexpr bool W16 = (RBL_G44_W16 && !PAIR && AG == 2) || DUO;
  // the basis loads: a wave-uniform base (the panel, the chunk's rows) plus an unsigned 32-bit
  // lane offset, so they can issue in the saddr form without per-load 64-bit address VALU
  const double* wpan = W.base + (int64_t)__builtin_amdgcn_readfirstlane(PAIR || DUO ? 2 * j : j) * W.stride;
  const unsigned wlo = (unsigned)((W16 ? 2 * (lane & 15) : (lane & 15)) + q * B);
  const int64_t wag = PAIR ? W.stride : 16;
  auto shift = [&](int64_t rc0) -> int64_t { return rc0 < r_end - kG44Rows ? rc0 : r_end - kG44Rows; };
  auto load_x = [&](int64_t rc0, double (&xr)[EPT]) {
    const double* p = xsl + shift(rc0) * B;
#pragma unroll
    for (int v = 0; v < EPT; ++v) xr[v] = p[v];
  };
  auto store_x = [&](int buf, int64_t rc0, const double (&xr)[EPT]) {
    const int64_t row = shift(rc0) + xrow;
    const bool ok = row >= rc0 && row < r_end;
#pragma unroll
    for (int v = 0; v < EPT; ++v) xs[buf][xrow * LD + perm8(xcol + v)] = ok ? xr[v] : 0.0;
  };
  // GL: this wave's lines of the chunk; lane -> slot lane / (KC / 2), column 2 (lane % (KC / 2))
  const double* gl_src[GL ? GLn::NL / kG44Waves : 1];
  if constexpr (GL) {
    const int col = 2 * (lane % (KC / 2));
    const double* xp = col >= B ? X.ptr[NX - 1] : X.ptr[0];
#pragma unroll
    for (int i = 0; i < GLn::NL / kG44Waves; ++i)
      gl_src[i] = xp + (int64_t)GLn::row(wave * (GLn::NL / kG44Waves) + i, lane / (KC / 2)) * B + col % B;
  }
  auto dma_x = [&](int buf, int64_t rc0) {
    const int64_t rb = shift(rc0) * B;
#pragma unroll
    for (int i = 0; i < GLn::NL / kG44Waves; ++i)
      __builtin_amdgcn_global_load_lds((glb_vptr)(gl_src[i] + rb),
                                       (lds_vptr)(xs[buf] + (wave * (GLn::NL / kG44Waves) + i) * kLine),
                                       16, 0, 0);
  };
  auto load_a = [&](int64_t rc0, double (&ar)[KS][AG]) {
    const double* p = wpan + shift(rc0) * B;  // uniform
    if constexpr (DUO) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const d2v v = ldw(reinterpret_cast<const d2v*>(p + h * W.stride + (wlo + (unsigned)(4 * ks * B))));
          ar[ks][2 * h] = v.x;
          ar[ks][2 * h + 1] = v.y;
        }
    } else if constexpr (W16) {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) {
        const d2v v = ldw(reinterpret_cast<const d2v*>(p + (wlo + (unsigned)(4 * ks * B))));
        ar[ks][0] = v.x;
        ar[ks][AG - 1] = v.y;
      }
    } else {
#pragma unroll
      for (int ks = 0; ks < KS; ++ks)
#pragma unroll
        for (int ag = 0; ag < AG; ++ag) ar[ks][ag] = ldw(p + wag * ag + (wlo + (unsigned)(4 * ks * B)));
    }
  };

  auto mma = [&](const double* xbuf, const double (&acur)[KS][AG]) {
    const double* xb = GL ? xbuf + 8 * cp0 + q * kLine + 2 * (lane & 3) : xbuf + 8 * cp0;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
#pragma unroll
      for (int cp = 0; cp < CGP / 2; ++cp) {  // column groups 2cp, 2cp+1 in one 16-B read
        const d2v bf = GL ? *reinterpret_cast<const d2v*>(xb + GLn::off(4 * ks) + 8 * cp)
                          : *reinterpret_cast<const d2v*>(xb + (4 * ks + q) * LD + 8 * cp + 2 * (lane & 3));
#pragma unroll
        for (int ag = 0; ag < AG; ++ag) {
          acc[ag][2 * cp] = mfma4(acur[ks][ag], bf.x, acc[ag][2 * cp]);
          acc[ag][2 * cp + 1] = mfma4(acur[ks][ag], bf.y, acc[ag][2 * cp + 1]);
        }
      }
    }
  };

  // GL: the loop covers whole chunks only; a last partial chunk (shifted back, rows below
  // rc0 zeroed) goes through the register path after it
  // cs: rows from one chunk of this split to its next (16: a contiguous split; 16 x splits:
  // interleaved, every split's k-th chunk adjacent to the others' so the chip sweeps the basis
  // front to back).  GL counts whole chunks only (a partial last chunk goes through the tail).
  const int64_t nchunks =
      r_end > r_begin ? (GL ? (r_end - r_begin >= kG44Rows ? (r_end - r_begin - kG44Rows) / cs + 1 : 0)
                            : (r_end - r_begin + cs - 1) / cs)
                      : 0;
  double xr[EPT];
  constexpr int PFD = B == 16 ? RBL_G44_PF16 : RBL_G44_PF;
  static_assert(PFD >= 1 && PFD <= 3, "prefetch distance");
  if constexpr (PFD == 3) {
    // four rotating register sets, the loop unrolled by 4
    double a0[KS][AG], a1[KS][AG], a2[KS][AG], a3[KS][AG];
    if (nchunks > 0) {
      if constexpr (GL) {
        dma_x(0, r_begin);
      } else {
        load_x(r_begin, xr);
        store_x(0, r_begin, xr);
      }
      load_a(r_begin, a0);
      load_a(r_begin + cs, a1);
      load_a(r_begin + 2 * cs, a2);
    }
    __syncthreads();
    auto step = [&](int64_t c, const double (&acur)[KS][AG], double (&afut)[KS][AG]) {
      const int64_t rc0 = r_begin + c * cs;
      if constexpr (GL) dma_x((int)((c + 1) & 1), rc0 + cs);
      else load_x(rc0 + cs, xr);
      load_a(rc0 + 3 * cs, afut);
      if (active && c < nchunks) mma(xs[c & 1], acur);
      if constexpr (!GL) store_x((int)((c + 1) & 1), rc0 + cs, xr);
      __syncthreads();
    };
    for (int64_t c = 0; c < nchunks; c += 4) {
      step(c, a0, a3);
      step(c + 1, a1, a0);
      step(c + 2, a2, a1);
      step(c + 3, a3, a2);
    }
    if constexpr (GL) {
      const int64_t rc0 = r_begin + nchunks * cs;
      if (rc0 < r_end) {
        load_x(rc0, xr);
        load_a(rc0, a0);
#pragma unroll
        for (int v = 0; v < EPT; ++v) {
          const int64_t row = shift(rc0) + xrow;
          xs[0][GLn::off(xrow) + xcol + v] = row >= rc0 ? xr[v] : 0.0;
        }
        __syncthreads();
        if (active) mma(xs[0], a0);
      }
    }
  } else if constexpr (PFD == 2) {
  // basis operands two chunks ahead in three rotating register sets (no copies: a copy of a
  // landing prefetch would make the wave wait for it one chunk early)
  double a0[KS][AG], a1[KS][AG], a2[KS][AG];
  if (nchunks > 0) {
    if constexpr (GL) {
      dma_x(0, r_begin);
    } else {
      load_x(r_begin, xr);
      store_x(0, r_begin, xr);
    }
    load_a(r_begin, a0);
    load_a(r_begin + cs, a1);
  }
  __syncthreads();
  auto step = [&](int64_t c, const double (&acur)[KS][AG], double (&afut)[KS][AG]) {
    const int64_t rc0 = r_begin + c * cs;
    if constexpr (GL) dma_x((int)((c + 1) & 1), rc0 + cs);
    else load_x(rc0 + cs, xr);
    load_a(rc0 + 2 * cs, afut);
    if (active && c < nchunks) mma(xs[c & 1], acur);  // no loads inside: vmcnt bookkeeping unaffected
    if constexpr (!GL) store_x((int)((c + 1) & 1), rc0 + cs, xr);
    __syncthreads();
  };
  for (int64_t c = 0; c < nchunks; c += 3) {
    step(c, a0, a2);
    step(c + 1, a1, a0);
    step(c + 2, a2, a1);
  }
  if constexpr (GL) {
    const int64_t rc0 = r_begin + nchunks * cs;
    if (rc0 < r_end) {  // every DMA has landed (closing barrier of the last step)
      load_x(rc0, xr);
      load_a(rc0, a0);
#pragma unroll
      for (int v = 0; v < EPT; ++v) {
        const int64_t row = shift(rc0) + xrow;
        xs[0][GLn::off(xrow) + xcol + v] = row >= rc0 ? xr[v] : 0.0;
      }
      __syncthreads();
      if (active) mma(xs[0], a0);
    }
  }
  } else {
  static_assert(!GL, "GL: PF = 2 only");
  double acur[KS][AG], anext[KS][AG];
  if (nchunks > 0) {
    load_x(r_begin, xr);
    store_x(0, r_begin, xr);
    load_a(r_begin, acur);
  }
  __syncthreads();
  for (int64_t c = 0; c < nchunks; ++c) {
    const int64_t rc0 = r_begin + c * cs;
    // unconditional (clamped on the last chunk): a uniform branch here would make the
    // waitcnt pass merge a no-load path and drain the prefetch before the MFMAs
    load_x(rc0 + cs, xr);
    if (!(RBL_REORTH_ABL & 1)) load_a(rc0 + cs, anext);
    if (active) mma(xs[c & 1], acur);  // idle waves (a 3-panel group) only help stage X
    // unconditional as well: a consumer under `if (more)` lets LLVM sink the loads into it
    // (after the MFMAs); on the last chunk this writes the dead spare buffer
    if (!(RBL_REORTH_ABL & 4)) store_x((int)((c + 1) & 1), rc0 + cs, xr);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks)
#pragma unroll
      for (int ag = 0; ag < AG; ++ag) acur[ks][ag] = anext[ks][ag];
    if (!(RBL_REORTH_ABL & 2)) __syncthreads();
  }
  }
  if (!active) return;
  const int KW = W.count * B;
  double* out = slab + (s * KW + (int64_t)j * WB) * KC + 4 * (2 * cp0);
  const int g = (lane >> 2) & 3;
#pragma unroll
  for (int ag = 0; ag < AG; ++ag)
#pragma unroll
    for (int cg = 0; cg < CGP; ++cg) {
      const int a = DUO   ? 32 * (ag >> 1) + 2 * (4 * g + (lane >> 4)) + (ag & 1)
                    : W16 ? 2 * (4 * g + (lane >> 4)) + ag
                          : 16 * ag + 4 * g + (lane >> 4);
      const int cc = GL ? 8 * (cg >> 1) + 2 * (lane & 3) + (cg & 1) : 4 * cg + (lane & 3);
      out[(int64_t)a * KC + cc] = acc[ag][cg];
    }
}

template <int B, int NX, bool PAIR = false, bool GL = false, bool DUO = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(DUO ? RBL_G44_DUO_WPE : B == 16 ? RBL_G44_WPE16 : RBL_G44_WPE))) void k_gram44(
    int64_t nrows, PanelRun W, Panels X, double* slab, int npg, int64_t rows_per, const int* skip) {
  if (skip && *skip) return;
  constexpr int KC = NX * B;
  constexpr int CG = KC / 4;
  constexpr int NPH2 = CG / 2 >= 2 ? 2 : 1;
  constexpr int NPH4 = CG / 2 >= 4 ? 4 : NPH2;
  constexpr int XS = GL ? 2 * G44Lines<KC>::NL * kLine : 2 * kG44Rows * (KC + 8);
  __shared__ __attribute__((aligned(16))) double xs[XS];
  // XCD-aware mapping: the npg workgroups of one row split share blockIdx % 8 (one XCD under
  // round-robin dispatch) and are consecutive there, so X is fetched once per XCD L2.
  const int bid = blockIdx.x;
  const int xcd = bid & 7, t = bid >> 3;
  const int pg = t % npg;
  const int64_t s = (int64_t)(t / npg) * 8 + xcd;
  // RBL_G44_INTER(16): interleaved splits (split s takes chunks s, s + S, ...; S = splits)
  constexpr bool kInter = B == 16 ? RBL_G44_INTER16 : RBL_G44_INTER;
  const int64_t S = gridDim.x / npg;
  const int64_t r_begin = kInter ? s * kG44Rows : s * rows_per;
  const int64_t r_end = kInter ? nrows : (r_begin + rows_per < nrows ? r_begin + rows_per : nrows);
  const int64_t cs = kInter ? S * kG44Rows : kG44Rows;
  const int rem = (PAIR || DUO ? W.count / 2 : W.count) - pg * kG44Waves;
  const int r = rem < kG44Waves ? rem : kG44Waves;  // panels in this group (workgroup-uniform)
  if (r >= 3) gram44_body<B, NX, 1, PAIR, GL, DUO>(r_begin, r_end, cs, s, pg, r, W, X, slab, xs);
  else if (r == 2) gram44_body<B, NX, NPH2, PAIR, GL, DUO>(r_begin, r_end, cs, s, pg, r, W, X, slab, xs);
  else gram44_body<B, NX, NPH4, PAIR, GL, DUO>(r_begin, r_end, cs, s, pg, r, W, X, slab, xs);
}

bool gram44_ok(int64_t nrows, int nW, int w, int xcount, int xw) {
  return nrows >= kG44Rows && nW >= 2 && (w == 16 || w == 32) && xw == w &&
         (xcount == 1 || xcount == 2);
}

// Splits: between one and two per resident workgroup slot (3 x CUs .. 6 x CUs), at most one
// per RBL_G44_SPLIT_ROWS rows.  Short splits balance the launch's tail; below a few thousand
// rows each, the per-split partial (slab write + reduction) costs more than that saves.
// Measured (tools/reorth_probe, profiles/r03_gram_splits_ab.log): 6 x CUs splits -1.2 % at
// n = 1e7 (6.5 k rows each), but 976 splits at n = 4e6 (4.1 k rows) +1.7 % and 6 x CUs at
// 1.25e6 +2.3 %; a cap at two waves of workgroups +6 %.  So >= 6 k rows per split.
#ifndef RBL_G44_SPLIT_ROWS
#define RBL_G44_SPLIT_ROWS 6144
#endif
int gram44_splits(int64_t nrows, int nW, int w) {
  (void)nW;
  const int64_t wpe = w == 16 ? RBL_G44_WPE16 : RBL_G44_WPE;
  const int64_t slots8 = wpe * window_grid() / 8;  // XCD mapping: multiples of 8
  int64_t s8 = nrows / (8 * (int64_t)RBL_G44_SPLIT_ROWS);
  s8 = std::min(std::max(s8, slots8), 2 * slots8);
  const int64_t max_s8 = (nrows + 8 * 128 - 1) / (8 * 128);  // each split >= 128 rows
  if (s8 > max_s8) s8 = max_s8;
  if (s8 < 1) s8 = 1;
  return (int)(s8 * 8);
}

template <int B, int NX, bool PAIR = false, bool DUO = false>
static void launch_gram44(int64_t nrows, const PanelRun& W, const Panels& X, double* slab,
                          int splits, const int* skip, hipStream_t st) {
  const int units = PAIR || DUO ? W.count / 2 : W.count;
  const int npg = (units + kG44Waves - 1) / kG44Waves;
  int64_t rows_per = (nrows + splits - 1) / splits;
  rows_per = (rows_per + kG44Rows - 1) / kG44Rows * kG44Rows;
  constexpr bool kGL = (B == 16 ? RBL_G44_GLDS16 : RBL_G44_GLDS) && (B == 16 ? RBL_G44_PF16 : RBL_G44_PF) >= 2 && kG44Rows == 16 && (NX * B == 32 || NX * B == 64);
  bool gl = kGL;
  for (int t = 0; t < X.count; ++t) gl &= reinterpret_cast<uintptr_t>(X.ptr[t]) % 16 == 0;
  if (gl)
    hipLaunchKernelGGL((k_gram44<B, NX, PAIR, kGL, DUO>), dim3(npg * splits), dim3(256), 0, st, nrows, W, X,
                       slab, npg, rows_per, skip);
  else
    hipLaunchKernelGGL((k_gram44<B, NX, PAIR, false, DUO>), dim3(npg * splits), dim3(256), 0, st, nrows, W,
                       X, slab, npg, rows_per, skip);
}

void gram44_partial(int64_t nrows, const PanelRun& W, const Panels& X, double* slab, int splits,
                    const int* skip, hipStream_t st) {
  if (W.w == 32) {
#ifdef RBL_VARIANTS
    // (variants build only) RBL_G44_DUO=1: panel pairs per wave (A/B; see gram44_body)
    static const bool duo_ok = [] {
      const char* e = getenv("RBL_G44_DUO");
      return e && atoi(e) != 0;
    }();
    if (duo_ok && X.count == 2 && W.count % 2 == 0)
      return launch_gram44<32, 2, false, true>(nrows, W, X, slab, splits, skip, st);
#endif
    if (X.count == 2) return launch_gram44<32, 2>(nrows, W, X, slab, splits, skip, st);
    return launch_gram44<32, 1>(nrows, W, X, slab, splits, skip, st);
  }
  // b = 16 with an even panel count (partial reorth: i - 2 panels at even i): panel pairs
#ifdef RBL_VARIANTS
  static const bool pair_ok = [] {  // RBL_G44_PAIR=0: one panel per wave (A/B)
    const char* e = getenv("RBL_G44_PAIR");
    return !e || atoi(e) != 0;
  }();
#else
  constexpr bool pair_ok = true;
#endif
  if (pair_ok && W.count % 2 == 0) {
    if (X.count == 2) return launch_gram44<16, 2, true>(nrows, W, X, slab, splits, skip, st);
    return launch_gram44<16, 1, true>(nrows, W, X, slab, splits, skip, st);
  }
  if (X.count == 2) return launch_gram44<16, 2>(nrows, W, X, slab, splits, skip, st);
  return launch_gram44<16, 1>(nrows, W, X, slab, splits, skip, st);
}

// ----------------------------------------------------------------------------------------
// Y = beta Y + alpha X C: 4 waves x 32 rows per workgroup, C staged in LDS 32 k at a time,
// A operands read 2 k per 16-B load (k permuted consistently in A and B), next chunk's A
// prefetched while the current one computes.
// ----------------------------------------------------------------------------------------
constexpr int kT44Rows = 32;   // rows per wave (k_tsmm44)
#ifndef RBL_T44_NRT
#define RBL_T44_NRT 2
#endif
constexpr int kT44fNrt = RBL_T44_NRT;      // 16-row tiles per wave (k_tsmm44f)
constexpr int kT44fRows = 16 * kT44fNrt;   // rows per wave (k_tsmm44f)
constexpr int kT44K = 32;      // k per chunk

template <int B, int KYP, bool F32X = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(B == 16 ? RBL_T44_WPE16 : 3))) void k_tsmm44(int64_t nrows, PanelRun X, const double* __restrict__ C,
                                                int ldc, int KY, Panels Y, double alpha, double beta,
                                                const int* skip) {
  if (skip && *skip) return;
  constexpr int CG = KYP / 4;
  constexpr int LDC = KYP + 8;  // lane-group rows differ by 2: LDC = 8 mod 16 (see k_gram44)
  __shared__ __attribute__((aligned(16))) double cs[2][kT44K * LDC];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int q = lane >> 4;
  const int64_t r0 = ((int64_t)blockIdx.x * 4 + wave) * kT44Rows;
  const int K = X.count * B;
  const int nch = (K + kT44K - 1) / kT44K;

  double acc[2][CG];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt)
#pragma unroll
    for (int cg = 0; cg < CG; ++cg) acc[rt][cg] = 0.0;

  // Y rows for beta != 0, row-major 16 B per lane (element e = 2 lane + 128 m of each
  // 16-row tile), loaded before the k-loop so their latency hides behind it
  constexpr int kYPer = 16 * KYP / 128;
  constexpr bool kPrefY = KYP <= 32;  // b x b updates (one k-chunk); long-K runs load Y late
  d2v yold[2][kYPer];
  auto load_y = [&](int rt, int m) -> d2v {
    const int e = 2 * lane + 128 * m, row = e / KYP, c = e % KYP;
    int64_t r = r0 + 16 * rt + row;
    r = r < nrows ? r : nrows - 1;
    const int cc = c < KY ? c : 0;
    const int t = cc / Y.w;
    return *reinterpret_cast<const d2v*>(Y.ptr[t] + r * Y.w + (cc - t * Y.w));
  };
  if (kPrefY && beta != 0.0) {
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int m = 0; m < kYPer; ++m) yold[rt][m] = load_y(rt, m);
  }

  // A: rows r0 + 16 rt + (lane&15); k = k0 + 8 h + 2 q + v, h in [0,4), v in {0,1}
  // Prefetch loads are unconditional (clamped addresses) so each chunk issues the same VMEM
  // ops and the vmcnt waits count only the chunk consumed.  Rows past nrows compute garbage
  // that is never stored; k past K reads a valid panel but meets zeroed C rows (zeroed at
  // the LDS store).
  int64_t arow[2];
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
    const int64_t r = r0 + 16 * rt + (lane & 15);
    arow[rt] = r < nrows ? r : nrows - 1;
  }
  auto load_a = [&](int ch, d2v (&ar)[2][4]) {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const int k0 = ch * kT44K + 8 * h + 2 * q;
      const int k = k0 < K ? k0 : K - 2;
      const int pan = k / B;
      const int col = k - pan * B;
      if constexpr (F32X) {  // fp32 basis: two floats widened exactly
        const float* xp = X.base32 + (int64_t)pan * X.stride + col;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
          const float2 f = *reinterpret_cast<const float2*>(xp + arow[rt] * B);
          ar[rt][h].x = (double)f.x;
          ar[rt][h].y = (double)f.y;
        }
      } else {
        const double* xp = X.base + (int64_t)pan * X.stride + col;
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) ar[rt][h] = ldw(reinterpret_cast<const d2v*>(xp + arow[rt] * B));
      }
    }
  };
  // C chunk: 32 x KYP, 256 threads; element e -> (k = e / KYP, c = e % KYP)
  constexpr int CEPT = kT44K * KYP / 256;
  auto load_c = [&](int ch, double (&cr)[CEPT]) {
#pragma unroll
    for (int v = 0; v < CEPT; ++v) {
      const int e = tid + v * 256;
      const int k = ch * kT44K + e / KYP, c = e % KYP;
      const int kc = k < K ? k : K - 1, cc = c < KY ? c : KY - 1;
      cr[v] = C[(int64_t)kc * ldc + cc];
    }
  };
  auto store_c = [&](int buf, int ch, const double (&cr)[CEPT]) {
#pragma unroll
    for (int v = 0; v < CEPT; ++v) {
      const int e = tid + v * 256;
      const int k = ch * kT44K + e / KYP, c = e % KYP;
      cs[buf][(e / KYP) * LDC + perm8(e % KYP)] = (k < K && c < KY) ? cr[v] : 0.0;
    }
  };

  d2v acur[2][4], anext[2][4];
  double cr[CEPT];
  load_c(0, cr);
  store_c(0, 0, cr);
  load_a(0, acur);
  __syncthreads();
  for (int ch = 0; ch < nch; ++ch) {
    load_c(ch + 1, cr);  // unconditional, clamped (see k_gram44)
    load_a(ch + 1, anext);
    const double* cb = cs[ch & 1] + 2 * q * LDC + 2 * (lane & 3);
#pragma unroll
    for (int hv = 0; hv < 8; ++hv) {
      const int h = hv >> 1, v = hv & 1;
      const double* cr0 = cb + (8 * h + v) * LDC;
#pragma unroll
      for (int cp = 0; cp < CG / 2; ++cp) {  // column groups 2cp, 2cp+1 in one 16-B read
        const d2v bf = *reinterpret_cast<const d2v*>(cr0 + 8 * cp);
#pragma unroll
        for (int rt = 0; rt < 2; ++rt) {
          acc[rt][2 * cp] = mfma4(acur[rt][h][v], bf.x, acc[rt][2 * cp]);
          acc[rt][2 * cp + 1] = mfma4(acur[rt][h][v], bf.y, acc[rt][2 * cp + 1]);
        }
      }
    }
    store_c((ch + 1) & 1, ch + 1, cr);  // unconditional (see k_gram44)
#pragma unroll
    for (int rt = 0; rt < 2; ++rt)
#pragma unroll
      for (int h = 0; h < 4; ++h) acur[rt][h] = anext[rt][h];
    __syncthreads();
  }
  // epilogue: the D-layout tile goes through LDS (the C buffers are free after the loop's
  // last barrier) so Y is read and written row-major, 16 B per lane, fully coalesced; Y was
  // prefetched before the k-loop.  Column c of staged row r sits at c ^ (4 ((r >> 2) & 3)):
  // the four row quads a ds_write_b64 lane group covers land 8 banks apart.
  double* ot = &cs[0][0] + wave * 16 * KYP;
  const int g = (lane >> 2) & 3;
#pragma unroll
  for (int rt = 0; rt < 2; ++rt) {
#pragma unroll
    for (int cg = 0; cg < CG; ++cg)
      ot[(4 * g + q) * KYP + ((4 * cg + (lane & 3)) ^ (4 * g))] = alpha * acc[rt][cg];
#pragma unroll
    for (int m = 0; m < kYPer; ++m) {
      const int e = 2 * lane + 128 * m, row = e / KYP, c = e % KYP;
      const int64_t r = r0 + 16 * rt + row;
      d2v v = *reinterpret_cast<const d2v*>(ot + row * KYP + (c ^ (4 * ((row >> 2) & 3))));
      if (r < nrows && c < KY) {
        const int t = c / Y.w;
        d2v* yp = reinterpret_cast<d2v*>(const_cast<double*>(Y.ptr[t]) + r * Y.w + (c - t * Y.w));
        if (beta != 0.0) v += beta * (kPrefY ? yold[rt][m] : load_y(rt, m));
        *yp = v;
      }
    }
  }
}

// Fast path of k_tsmm44 for the partial-reorth update (64 output columns, K a multiple of 32,
// nrows >= 32): every address is a wave-uniform base plus a lane constant, so the k-loop runs
// no per-load VALU (k_tsmm44 spent ~0.6 VALU per MFMA on clamps and 64-bit address math, and
// on gfx950 fp64 MFMA does not co-execute with VALU).  A wave whose 32 rows pass nrows computes
// the last 32 rows instead and stores only its own.
// KC: k per chunk (C chunk staged in LDS per chunk); PF: chunks of basis operands in flight
// ahead of the MFMAs (PF = 2: three rotating register sets, the loop unrolled by 3).
#ifndef RBL_T44_KC
#define RBL_T44_KC 32
#endif
#ifndef RBL_T44_PF
#define RBL_T44_PF 1
#endif
// XG (Y = [Q_i | Q_{i-1}], 32 columns each): each workgroup also forms Q_{i-1}^T Q_i over its
// final rows (16x16x4 MFMAs from the output stage) into xslab[blockIdx] (one 32 x 32 partial
// per 128-row tile) — the local-reorth coefficient of the same step (RBL_gpu.jl:87), formed
// while the partial-reorth update writes the blocks instead of in another pass over both.
// GL: the C chunk is staged by LDS-DMA (global_load_lds_dwordx4: no VGPRs, no ds_write) into
// 1-KiB lines padded to 1088 B; a C row (KYP doubles) lies whole in one line slot, rows placed
// so that the 4 rows one ds_read_b128 touches (k = 8h + v + 2q, q = 0..3) sit in 4 lines:
// conflict-free reads with a lane offset q * 1088 + 16 (lane & 3) and compile-time rest.  Lane
// (lane & 3) then reads columns 8cp + 2(lane & 3) + {0, 1} (GL = false: perm8 order, columns
// 4(2cp) + (lane & 3) and 4(2cp+1) + (lane & 3)); only the accumulator -> column map differs,
// every output sums the same products in the same order.  Needs C 16-B aligned, ldc even.
// Off by default: bit-identical, VALU per MFMA 0.273 -> 0.220, but MFMA busy 0.827 -> 0.802 and
// 0.8 % slower over 5 alternating probe reps (profiles/r03_pmc_reorth_glds.txt)
#ifndef RBL_T44_GLDS
#define RBL_T44_GLDS 0
#endif
template <int KYP>
struct T44Lines {
  static constexpr int RPL = 1024 / (8 * KYP);  // C rows per 1-KiB line (2 or 4)
  static constexpr int LINE = kLine;            // doubles per padded line (1088 B)
  // row R = 8h + v + 2q of a chunk -> (line, slot); inverse for the DMA writer
  __device__ static constexpr int line(int R) {
    return RPL == 2 ? R >> 1 : 4 * (R >> 4) + ((R >> 1) & 3);
  }
  __device__ static constexpr int slot(int R) { return RPL == 2 ? R & 1 : (R & 1) + 2 * ((R >> 3) & 1); }
  __device__ static constexpr int row(int L, int s) {
    return RPL == 2 ? 2 * L + s : 16 * (L >> 2) + 2 * (L & 3) + (s & 1) + 8 * (s >> 1);
  }
  __device__ static constexpr int off(int R) { return line(R) * LINE + slot(R) * KYP; }
};

template <int B, int KC = RBL_T44_KC, int PF = RBL_T44_PF, bool XG = false, int KYP = 64, bool GL = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(kT44fNrt == 2 ? 3 : 2))) void k_tsmm44f(
    int64_t nrows, PanelRun X, const double* __restrict__ C, int ldc, Panels Y, double alpha,
    double beta, const int* skip, double* __restrict__ xslab) {
  if (skip && *skip) return;
  constexpr int CG = KYP / 4, LDC = KYP + 8;
  constexpr int YW = KYP / 2, NT = YW / 16;  // XG: Y = [Q_i | Q_{i-1}], YW columns each
  constexpr int NH = KC / 8;  // 16-B A loads per row tile per chunk
  constexpr int CEPT = KC * KYP / 256;
  using TL = T44Lines<KYP>;
  constexpr int NL = KC / TL::RPL;  // GL: lines per chunk
  static_assert(!GL || (NL % 4 == 0 && KC % 16 == 0), "GL chunk shape");
  constexpr int CB = GL ? NL * TL::LINE : KC * LDC;  // doubles per C buffer
  constexpr int CS = 2 * CB > 4 * 16 * KYP ? 2 * CB : 4 * 16 * KYP;  // + epilogue stage
  __shared__ __attribute__((aligned(16))) double cs_raw[CS];
  double(*cs)[CB] = reinterpret_cast<double(*)[CB]>(cs_raw);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int q = lane >> 4;
  const int nch = X.count * B / KC;
    // one 128-row tile per workgroup, or (XG) persistent over tiles
  auto tile_body = [&](int64_t tile) {
  typedef double d4x __attribute__((ext_vector_type(4)));
  d4x gx[XG ? NT : 1][XG ? NT : 1];
  if constexpr (XG) {
#pragma unroll
    for (int it = 0; it < NT; ++it)
#pragma unroll
      for (int jt = 0; jt < NT; ++jt) gx[it][jt] = d4x{0.0, 0.0, 0.0, 0.0};
  }
  constexpr int NRT = kT44fNrt;
  const int64_t r0 = (tile * 4 + wave) * kT44fRows;
  const int64_t rw = r0 + kT44fRows <= nrows ? r0 : nrows - kT44fRows;  // wave-uniform

  double acc[NRT][CG];
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
    for (int cg = 0; cg < CG; ++cg) acc[rt][cg] = 0.0;

  // A: rows rw + 16 rt + (lane&15), k = KC ch + 8 h + 2 q + v
  // every load is a wave-uniform base (SGPRs) plus an unsigned 32-bit lane offset, so it can
  // issue in the saddr form with no per-load 64-bit address VALU
  const unsigned aoff0 = (unsigned)((lane & 15) * B + 2 * q);
  auto load_a = [&](int ch, d2v (&ar)[NRT][NH]) {
    const int chc = ch < nch ? ch : nch - 1;
#pragma unroll
    for (int h = 0; h < NH; ++h) {
      const int kk = KC * chc + 8 * h;
      const double* xb = X.base + (int64_t)(kk / B) * X.stride + rw * B + (kk % B);
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt)
        ar[rt][h] = *reinterpret_cast<const d2v*>(xb + (aoff0 + (unsigned)(16 * rt * B)));
    }
  };
  // C chunk element tid + 256 v: row KC chc + tid / KYP + (256 / KYP) v, column tid % KYP
  constexpr int CRS = 256 / KYP;
  const unsigned coff = (unsigned)((tid / KYP) * ldc + tid % KYP);
  auto load_c = [&](int ch, double (&cr)[CEPT]) {
    const int chc = ch < nch ? ch : nch - 1;
#pragma unroll
    for (int v = 0; v < CEPT; ++v) {
      const double* cb = C + (int64_t)(KC * chc + CRS * v) * ldc;  // uniform
      cr[v] = cb[coff];
    }
  };
  const int cso = (tid / KYP) * LDC + perm8(tid % KYP);
  auto store_c = [&](int buf, const double (&cr)[CEPT]) {
#pragma unroll
    for (int v = 0; v < CEPT; ++v) cs[buf][cso + CRS * v * LDC] = cr[v];
  };
  // GL: this wave's NL / 4 lines of chunk ch; lane -> slot lane / (KYP / 2), pair lane % (KYP / 2)
  // (lane offsets are loop-invariant: a uniform chunk base plus a 32-bit lane offset per line)
  int gl_off[GL ? NL / 4 : 1];
  if constexpr (GL) {
    const int gl_slot = lane / (KYP / 2), gl_pair = lane % (KYP / 2);
#pragma unroll
    for (int i = 0; i < NL / 4; ++i) gl_off[i] = TL::row(wave * (NL / 4) + i, gl_slot) * ldc + 2 * gl_pair;
  }
  auto dma_c = [&](int buf, int ch) {
    const int chc = ch < nch ? ch : nch - 1;
    const double* cbase = C + (int64_t)KC * chc * ldc;
#pragma unroll
    for (int i = 0; i < NL / 4; ++i) {
      const int L = wave * (NL / 4) + i;
      __builtin_amdgcn_global_load_lds((glb_vptr)(cbase + gl_off[i]), (lds_vptr)(cs[buf] + L * TL::LINE), 16, 0, 0);
    }
  };
  auto mfmas = [&](int ch, const d2v (&acur)[NRT][NH]) {
    const double* cb = GL ? cs[ch & 1] + q * TL::LINE + 2 * (lane & 3)
                          : cs[ch & 1] + 2 * q * LDC + 2 * (lane & 3);
#pragma unroll
    for (int hv = 0; hv < 2 * NH; ++hv) {
      const int h = hv >> 1, v = hv & 1;
      const double* cr0 = cb + (GL ? TL::off(8 * h + v) : (8 * h + v) * LDC);
#pragma unroll
      for (int cp = 0; cp < CG / 2; ++cp) {
        const d2v bf = *reinterpret_cast<const d2v*>(cr0 + 8 * cp);
#pragma unroll
        for (int rt = 0; rt < NRT; ++rt) {
          acc[rt][2 * cp] = mfma4(acur[rt][h][v], bf.x, acc[rt][2 * cp]);
          acc[rt][2 * cp + 1] = mfma4(acur[rt][h][v], bf.y, acc[rt][2 * cp + 1]);
        }
      }
    }
  };

  double cr[CEPT];
  if constexpr (GL) {
    dma_c(0, 0);
  } else {
    load_c(0, cr);
    store_c(0, cr);
  }
  if constexpr (PF >= 2) {
    static_assert(!GL, "GL: PF = 1 only");
    d2v a0[NRT][NH], a1[NRT][NH], a2[NRT][NH];
    load_a(0, a0);
    load_a(1, a1);
    __syncthreads();
    auto step = [&](int ch, const d2v (&acur)[NRT][NH], d2v (&afut)[NRT][NH]) {
      load_c(ch + 1, cr);
      load_a(ch + 2, afut);
      if (ch < nch) mfmas(ch, acur);  // no loads inside: the vmcnt bookkeeping is unaffected
      store_c((ch + 1) & 1, cr);
      __syncthreads();
    };
    for (int ch = 0; ch < nch; ch += 3) {
      step(ch, a0, a2);
      step(ch + 1, a1, a0);
      step(ch + 2, a2, a1);
    }
  } else if constexpr (GL) {
    // two register sets swapped by a 2-unrolled loop (no copies); the DMA into the other
    // buffer (last read before the previous barrier) lands by the vmcnt(0) of this step's
    // closing barrier, before any wave reads it
    d2v a0[NRT][NH], a1[NRT][NH];
    load_a(0, a0);
    __syncthreads();
    auto step = [&](int ch, const d2v (&acur)[NRT][NH], d2v (&anext)[NRT][NH]) {
      dma_c((ch + 1) & 1, ch + 1);
      load_a(ch + 1, anext);
      if (ch < nch) mfmas(ch, acur);  // no loads inside: the vmcnt bookkeeping is unaffected
      __syncthreads();
    };
    for (int ch = 0; ch < nch; ch += 2) {
      step(ch, a0, a1);
      step(ch + 1, a1, a0);
    }
  } else {
    d2v acur[NRT][NH], anext[NRT][NH];
    load_a(0, acur);
    __syncthreads();
    for (int ch = 0; ch < nch; ++ch) {
      load_c(ch + 1, cr);
      if (!(RBL_REORTH_ABL & 1)) load_a(ch + 1, anext);
      mfmas(ch, acur);
      if (!(RBL_REORTH_ABL & 4)) store_c((ch + 1) & 1, cr);
#pragma unroll
      for (int rt = 0; rt < NRT; ++rt)
#pragma unroll
        for (int h = 0; h < NH; ++h) acur[rt][h] = anext[rt][h];
      if (!(RBL_REORTH_ABL & 2)) __syncthreads();
    }
  }
  // epilogue as k_tsmm44 (D layout -> LDS -> row-major 16-B stores); rows below r0 belong
  // to the previous wave (shifted last tile)
  double* ot = cs_raw + wave * 16 * KYP;
  const int g = (lane >> 2) & 3;
  constexpr int kYPer = 16 * KYP / 128;
  // a lane's stage column ce is the same for every m (128 % KYP == 0): its Y panel, column and
  // row base are hoisted (no per-store division or 64-bit multiply); rows r < nrows always
  // (rw + kT44fRows <= nrows), so "own" is row-in-tile >= r0 - rw
  constexpr int kRowStep = 128 / KYP;
  const int ce = (2 * lane) % KYP, rl = (2 * lane) / KYP;
  const int yt = ce >= Y.w ? 1 : 0;
  double* yb = const_cast<double*>(yt ? Y.ptr[Panels::kMax - 1] : Y.ptr[0]) + (ce - yt * Y.w) +
               (rw + rl) * Y.w;
  const int dskip = (int)(r0 - rw);
  const bool has_beta = beta != 0.0;
#pragma unroll
  for (int rt = 0; rt < NRT; ++rt) {
    if constexpr (GL) {
      // acc[rt][2cp + x] holds column 8cp + 2(lane & 3) + x
#pragma unroll
      for (int cp = 0; cp < CG / 2; ++cp)
        *reinterpret_cast<d2v*>(ot + (4 * g + q) * KYP + ((8 * cp + 2 * (lane & 3)) ^ (4 * g))) =
            d2v{alpha * acc[rt][2 * cp], alpha * acc[rt][2 * cp + 1]};
    } else {
#pragma unroll
      for (int cg = 0; cg < CG; ++cg)
        ot[(4 * g + q) * KYP + ((4 * cg + (lane & 3)) ^ (4 * g))] = alpha * acc[rt][cg];
    }
#pragma unroll
    for (int m = 0; m < kYPer; ++m) {
      const int row = rl + kRowStep * m;
      d2v v = *reinterpret_cast<const d2v*>(ot + row * KYP + (ce ^ (4 * ((row >> 2) & 3))));
      const bool own = 16 * rt + row >= dskip;
      if (own) {
        d2v* yp = reinterpret_cast<d2v*>(yb + (int64_t)((16 * rt + kRowStep * m) * Y.w));
        if (has_beta) v += beta * *yp;
        *yp = v;
      }
      if constexpr (XG)  // final values back into the stage (0 for rows this wave does not own)
        *reinterpret_cast<d2v*>(ot + row * KYP + (ce ^ (4 * ((row >> 2) & 3)))) = own ? v : d2v{0.0, 0.0};
    }
    if constexpr (XG) {
      // (Q_{i-1}^T Q_i)[16 it + .][16 jt + .] += sum over the 16 rows; row 4 s4 + q sits at
      // column c ^ (4 s4) of the stage
      const int li = lane & 15;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        const double* orow = ot + (4 * s4 + q) * KYP;
        double za[NT], yb[NT];
#pragma unroll
        for (int t2 = 0; t2 < NT; ++t2) {
          za[t2] = orow[(YW + 16 * t2 + li) ^ (4 * s4)];
          yb[t2] = orow[(16 * t2 + li) ^ (4 * s4)];
        }
#pragma unroll
        for (int it = 0; it < NT; ++it)
#pragma unroll
          for (int jt = 0; jt < NT; ++jt)
            gx[it][jt] = __builtin_amdgcn_mfma_f64_16x16x4f64(za[it], yb[jt], gx[it][jt], 0, 0, 0);
      }
    }
  }
  if constexpr (XG) {
    // the four waves' partials summed in LDS (fixed order), one 32 x 32 partial per workgroup
    __syncthreads();
    const int li = lane & 15;
    constexpr int G2 = YW * YW;
    double* gw = cs_raw + wave * G2;
#pragma unroll
    for (int it = 0; it < NT; ++it)
#pragma unroll
      for (int jt = 0; jt < NT; ++jt)
#pragma unroll
        for (int reg = 0; reg < 4; ++reg) gw[(16 * it + q + 4 * reg) * YW + 16 * jt + li] = gx[it][jt][reg];
    __syncthreads();
    double* out = xslab + tile * G2;
    for (int e = tid; e < G2; e += 256)
      out[e] = (cs_raw[e] + cs_raw[G2 + e]) + (cs_raw[2 * G2 + e] + cs_raw[3 * G2 + e]);
  }
  };
  tile_body(blockIdx.x);
}

// the epilogue stores Y row-major 16 B (two columns) per lane: Y panel widths must be even
bool tsmm44_ok(int xw, int ky, int yw) {
  return (xw == 16 || xw == 32) && ky >= 1 && ky <= 64 && yw % 2 == 0;
}

template <int B, int KYP, bool F32X = false>
static void launch_tsmm44(int64_t nrows, const PanelRun& X, const double* C, int ldc, int KY,
                          const Panels& Y, double alpha, double beta, const int* skip,
                          hipStream_t st) {
  const int64_t wgs = (nrows + 4 * kT44Rows - 1) / (4 * kT44Rows);
  hipLaunchKernelGGL((k_tsmm44<B, KYP, F32X>), dim3((unsigned)wgs), dim3(256), 0, st, nrows, X, C,
                     ldc, KY, Y, alpha, beta, skip);
}

void tsmm44_f32x(int64_t nrows, const PanelRun& X, const double* C, int ldc, const Panels& Y,
                 double alpha, double beta, hipStream_t st) {
  const int KY = Y.count * Y.w;
  if (X.w == 32) {
    if (KY <= 16) return launch_tsmm44<32, 16, true>(nrows, X, C, ldc, KY, Y, alpha, beta, nullptr, st);
    if (KY <= 32) return launch_tsmm44<32, 32, true>(nrows, X, C, ldc, KY, Y, alpha, beta, nullptr, st);
    return launch_tsmm44<32, 64, true>(nrows, X, C, ldc, KY, Y, alpha, beta, nullptr, st);
  }
  if (KY <= 16) return launch_tsmm44<16, 16, true>(nrows, X, C, ldc, KY, Y, alpha, beta, nullptr, st);
  if (KY <= 32) return launch_tsmm44<16, 32, true>(nrows, X, C, ldc, KY, Y, alpha, beta, nullptr, st);
  return launch_tsmm44<16, 64, true>(nrows, X, C, ldc, KY, Y, alpha, beta, nullptr, st);
}

int tsmm44_xg_grid(int64_t nrows) {
  // one partial per workgroup tile of k_tsmm44f (4 waves x kT44fRows rows)
  return (int)((nrows + 4 * kT44fRows - 1) / (4 * kT44fRows));
}

void tsmm44(int64_t nrows, const PanelRun& X, const double* C, int ldc, const Panels& Y,
            double alpha, double beta, const int* skip, hipStream_t st, double* xslab, int* xgrid) {
  if (xgrid) *xgrid = 0;
  const int KY = Y.count * Y.w;
#ifdef RBL_VARIANTS
  static const bool fast_ok = [] {  // RBL_TSMM44_FAST=0: the generic kernel (A/B)
    const char* e = getenv("RBL_TSMM44_FAST");
    return !e || atoi(e) != 0;
  }();
#else
  constexpr bool fast_ok = true;
#endif
  // fast path: 64 or 32 output columns, K a multiple of 32, Y not aliasing the X panels (a
  // wave writes its rows after the whole k-loop; the shifted last tile re-reads rows below it)
  bool alias = false;
  for (int t = 0; t < Y.count; ++t)
    alias |= Y.ptr[t] >= X.base && Y.ptr[t] < X.base + (int64_t)X.count * X.stride;
  // (KYP = 32 builds but stays off: at b = 16 the update is HBM-bound and the generic kernel
  // ran 4 % faster on C2, its cross-Gram form 6 % slower than the Gram pass it replaces —
  // tools/r02_c2_ab.sh; round 3 again 3 % faster on C2 and C3, profiles/r03_tsmm_fast32_ab.log)
#ifdef RBL_VARIANTS
  static const bool fast32 = [] {  // RBL_TSMM44_FAST32=1: the 32-column form too (A/B)
    const char* e = getenv("RBL_TSMM44_FAST32");
    return e && atoi(e) != 0;
  }();
#else
  constexpr bool fast32 = false;
#endif
  if (fast_ok && (KY == 64 || (KY == 32 && fast32)) && (X.count * X.w) % kT44K == 0 &&
      nrows >= kT44fRows && Y.w % 2 == 0 && !alias) {
    const int64_t wgs = (nrows + 4 * kT44fRows - 1) / (4 * kT44fRows);
    const bool xg = xslab && KY == 64 && Y.count == 2 && 2 * Y.w == KY;
    if (xg) *xgrid = (int)wgs;
    // LDS-DMA staging of C: 16-B aligned rows
    const bool gl = RBL_T44_GLDS && RBL_T44_PF == 1 && ldc % 2 == 0 &&
                    reinterpret_cast<uintptr_t>(C) % 16 == 0;
#define RBL_T44F(BB, XGG, KK)                                                                      \
  do {                                                                                              \
    if (gl)                                                                                         \
      hipLaunchKernelGGL((k_tsmm44f<BB, RBL_T44_KC, RBL_T44_PF, XGG, KK, RBL_T44_GLDS && RBL_T44_PF == 1>), \
                         dim3((unsigned)wgs), dim3(256), 0, st, nrows, X, C, ldc, Y, alpha, beta, skip, \
                         XGG ? xslab : nullptr);                                                    \
    else                                                                                            \
      hipLaunchKernelGGL((k_tsmm44f<BB, RBL_T44_KC, RBL_T44_PF, XGG, KK, false>), dim3((unsigned)wgs), \
                         dim3(256), 0, st, nrows, X, C, ldc, Y, alpha, beta, skip, XGG ? xslab : nullptr); \
  } while (0)
    if (KY == 64) {
      if (X.w == 32) { if (xg) RBL_T44F(32, true, 64); else RBL_T44F(32, false, 64); }
      else { if (xg) RBL_T44F(16, true, 64); else RBL_T44F(16, false, 64); }
    }
#ifdef RBL_VARIANTS
    else {
      if (X.w == 32) { if (xg) RBL_T44F(32, true, 32); else RBL_T44F(32, false, 32); }
      else { if (xg) RBL_T44F(16, true, 32); else RBL_T44F(16, false, 32); }
    }
#endif
#undef RBL_T44F
    return;
  }
  if (X.w == 32) {
    if (KY <= 16) return launch_tsmm44<32, 16>(nrows, X, C, ldc, KY, Y, alpha, beta, skip, st);
    if (KY <= 32) return launch_tsmm44<32, 32>(nrows, X, C, ldc, KY, Y, alpha, beta, skip, st);
    return launch_tsmm44<32, 64>(nrows, X, C, ldc, KY, Y, alpha, beta, skip, st);
  }
  if (KY <= 16) return launch_tsmm44<16, 16>(nrows, X, C, ldc, KY, Y, alpha, beta, skip, st);
  if (KY <= 32) return launch_tsmm44<16, 32>(nrows, X, C, ldc, KY, Y, alpha, beta, skip, st);
  return launch_tsmm44<16, 64>(nrows, X, C, ldc, KY, Y, alpha, beta, skip, st);
}

}  // namespace rbl
