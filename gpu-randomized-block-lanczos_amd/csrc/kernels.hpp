// kernels.hpp — host launchers for the gfx950 RBL kernels (implemented in *.hip).
#pragma once
#include "rbl_common.hpp"

namespace rbl {

// A list of n x w row-major panels ("blocks"): panel t starts at ptr[t] (t < count).
// Used for Krylov blocks (w = b), the pair [Q_i, Q_{i-1}] and the Ritz output (w = k).
struct Panels {
  static constexpr int kMax = 2;
  const double* ptr[kMax] = {nullptr, nullptr};
  int count = 0;
  int w = 0;              // width of each panel (leading dimension = w)
};
// Contiguous run of `count` panels of width w, panel j at base + j*stride (Krylov basis).
struct PanelRun {
  const double* base = nullptr;
  const float* base32 = nullptr;  // fp32 panels instead (tsmm44_f32x only)
  int64_t stride = 0;
  int count = 0;
  int w = 0;
};

// CSR rows [0,nrows) of the local slice; columns are global ids; Q row c lives at
// Qin + (c - col_off) * b.
// Device CSR arrays carry kCsrPad zero entries past nnz, and every n x b buffer an SpMM
// writes carries kRowPad spare rows: the band kernel's loads and stores run unguarded.
constexpr int64_t kCsrPad = 256;
constexpr int64_t kRowPad = 16;
// zeroed rows past the fp32 basis slots and the fp32 staging slot: the fp32 Gram's shifted
// chunks (reorth32.hip, up to this many rows) may read them when a slice has fewer rows
constexpr int64_t kRowPad32 = 32;

struct CsrDev {
  int64_t nrows = 0;
  int64_t nnz = 0;
  const int64_t* rowptr = nullptr;
  const int32_t* col = nullptr;
  const double* val = nullptr;
  // LDS-window metadata (16-row tiles): forward-filled min/max column per tile, and
  // whether every tile fits the window kernel's ring for b = 16 / b = 32.
  const int64_t* tile_cmin = nullptr;
  const int64_t* tile_cmax = nullptr;
  // per tile: e0, nnz, lo, hi (ring rows the tile adds), cmin, cmax, 0, 0
  const int64_t* tile_info = nullptr;
  int64_t ntiles = 0;
  int64_t tiles_per_wg = 0;
  // column-panel SpMM (spmm_panel.hip, b = 32): per block of panel_rows() local rows its first
  // and last panel of panel_width() Q rows (global ids); null: not applicable
  const int32_t* panel_blk = nullptr;   // per block: first / last panel, count offset (int64)
  const uint16_t* panel_cnt = nullptr;  // per block, panel and row: the row's entries there
  const uint32_t* panel_st = nullptr;   // ... and where they start (records from the block's base)
  const uint8_t* panel_col = nullptr;   // the records, panel-major within a block: column - panel
  const double* panel_val = nullptr;    //   base (one byte), value
  int64_t panel_nblk = 0;
  int panel_rpg = 4;         // rows per 16-lane group (blocks of 64 rpg rows): 4 or 8
  int panel_ch = 32;         // records per row and chunk load: 16 or 32
  bool panel_auto = false;   // the automatic choice takes it (else only when forced)
  bool window_ok16 = false;
  bool window_ok32 = false;
  bool band_ok16 = false;   // spmm_band.hip applicable (and dense enough to pay)
  bool band_ok32 = false;
  bool band_gram = false;   // every tile's own rows lie in its band window (ring-resident)
  bool band_pair = false;   // every tile-row pair (2p, 2p+1) has <= 253 nonzeros
  int64_t row0 = 0;         // global index of local row 0 (row-partitioned runs)
  // band kernel: per nonzero, its byte offset in the tile's dense LDS band
  // ((row % 16) * kBandLd + perm8(col - c16(tile))) * 8 (band_positions; kCsrPad entries past nnz)
  const uint16_t* band_pos = nullptr;
  // band-tile kernel (spmm_bt.hip): the CSR densified into MFMA-ordered 16-row tiles with
  // band groups NG = (2H+16)/16 (0: not applicable), and the Q rows the kernel may read
  // (global [q_lo, q_hi); other band rows read zrow, 32 zeros)
  const double* bt = nullptr;
  int bt_ng = 0;
  int64_t bt_tiles_per_wg = 0;
  int64_t q_lo = 0, q_hi = 0;
  const double* zrow = nullptr;
  // several ranks: the own rows [loc_lo, loc_hi) read straight from the block (fp64, or fp32
  // on the fp32-basis path) instead of from Qin, whose halo buffer then holds only the
  // neighbours' rows — no per-step copy of the local block.  Band-tile kernel only: spmm()
  // fails if another kernel would run with qloc set.
  const void* qloc = nullptr;
  int64_t loc_lo = 0, loc_hi = 0;
  // local reorth fused into the band-tile SpMM (RBL_OPT_FUSE bit 2, b = 32, dense tiles; one
  // rank or several — then each rank's edge rows are corrected before the halo exchange, by
  // spmm_bt_locfix_edges, and the SpMM leaves them as read): the kernel stages every Q ring row as Q_i - Q_{i-1} C (C = lfix_c, b x b on the
  // device; Q_{i-1} = the SpMM's Qprev) and writes the corrected own rows back into lfix_q
  // (the block Q_i) except the first and last H rows of each workgroup's range, which
  // neighbours read raw — spmm_bt_locfix_rest corrects those after the SpMM
  // (spmm_bt_locfix_ok: applicable; spmm_bt_locfix_edges: the rank-edge rows beforehand)
  const double* lfix_c = nullptr;
  double* lfix_q = nullptr;
  int* two_wave = nullptr;          // set to 1 when the two-waves-per-SIMD kernel (k_spmm_bt2) ran
  int64_t lfix_lo = 0, lfix_hi = 0;  // local rows still raw (several ranks: the rank's first and
                                     // last H rows were corrected before the halo exchange)
  // packed band tiles (bt_pack): per tile slot a header of bt_pack_words(NG) 8-B words (per
  // 1-KiB operand block the nonzero masks of element 0 / 1 of every lane, then the blocks'
  // uint16 start offsets + the tile's count, then the tile's first value index) and the
  // nonzeros per block: element 0 of the lanes, then element 1; null: the dense tiles `bt`
  const uint64_t* btp_hdr = nullptr;
  const double* btp_val = nullptr;
  // half band tiles (A symmetric, bt_half): groups NGL..NG-1 of every tile slot, and the
  // first NGL local tiles whole; replaces `bt`
  const double* bth = nullptr;
  const double* bte = nullptr;
  // segmented gather (spmm.hip variant 5): wave tasks (first row, info: > 0 rows of a packed
  // short-row task, < 0 -(slot+1) of a long-row segment), segment slots' first nonzero
  // (slot_k0, nslots + 1 entries), long rows with their first slot (lslot, nlong + 1), and a
  // scratch of nslots x 32 partial rows
  int64_t seg_ntasks = 0;
  const int64_t* seg_trow = nullptr;
  const int32_t* seg_tinfo = nullptr;
  const int64_t* seg_slot_k0 = nullptr;
  int64_t seg_nlong = 0;
  const int64_t* seg_lrow = nullptr;
  const int64_t* seg_lslot = nullptr;
  double* seg_scratch = nullptr;
  // column tiers of the segmented gather (RBL_SEG_TIERS; one rank): the nonzeros split by the
  // degree rank of their column into up to kMaxSegTiers CSRs of the same rows, each with its
  // own task table; the SpMM sweeps them in order, accumulating into U, so each sweep's Q-row
  // gathers come from a set that fits a cache level (hot rows: an XCD's L2)
  int seg_ntiers = 0;
  // several ranks: two tiers, the own columns [loc_lo, loc_hi) (tier 0, gathered from `qloc`,
  // the block itself, when set) and the halo columns (tier 1, from Qin): tier 0 runs while the
  // halo exchange is in flight; the stream waits for `seg_wait` (if set) before tier 1
  bool seg_split = false;
  hipEvent_t seg_wait = nullptr;
  struct Tier {
    const int64_t* rowptr = nullptr;
    const int32_t* col = nullptr;
    const double* val = nullptr;
    int64_t ntasks = 0, nlong = 0;
    const int64_t* trow = nullptr;
    const int32_t* tinfo = nullptr;
    const int64_t* slot_k0 = nullptr;
    const int64_t* lrow = nullptr;
    const int64_t* lslot = nullptr;
    double* scratch = nullptr;
  } seg_tier[3];
};
constexpr int kMaxSegTiers = 3;
constexpr int64_t kSegLen = 4096;   // nonzeros per long-row segment
constexpr int64_t kSegPack = 512;   // nonzeros per packed short-row task (<= 64 rows)

// --- rowop.hip ---------------------------------------------------------------------------
// Y' = beta Y + alpha X C (X, Y: n x b panels, C: b x b row-major, ldc) in one pass, and if
// slab != null the Gram Y'^T Y' as grid partials slab[grid][b][b] (reduce with reduce_slab).
// X may equal Y (in place).  b in {16, 32}.
bool rowgram_ok(int b);
int rowgram_grid(int64_t nrows, int per_cu = 2);
constexpr int kRowgramMaxPerCu = 4;  // rowgram_ex's grids stay <= rowgram_grid(nrows, this)
// X32 (optional): X read from fp32 instead (widened exactly).  Y32 (optional): Y' written to
// Y32 rounded to fp32 instead of Y — unless f64flag is non-null and *f64flag != 0 (device).
// tri: C is upper triangular (zeros below the diagonal), X fp64 — all-zero MFMA blocks skipped.
void rowgram(int64_t nrows, int b, const double* X, const double* C, int ldc, double* Y,
             double alpha, double beta, double* slab, int grid, const int* skip, hipStream_t s,
             const float* X32 = nullptr, float* Y32 = nullptr, const int* f64flag = nullptr,
             bool tri = false);
// The CholQR forms of the fused row op (b in {16, 32}, X fp64):
//   mode 1: slab <- Gram of X C (no store);  mode 2: Y = (X C) C2 (slab must be null);
//   Z != null (modes 0 and 2): slab2 <- per-workgroup partials of Z^T Y (grid x b x b).
// grid <= 0: as many persistent workgroups as the instantiation keeps resident (its register
// budget), reported in *grid_out.  Returns false for an unsupported combination.
struct RowOpArgs {
  const double* X = nullptr;
  const double* C = nullptr;
  int ldc = 0;
  double* Y = nullptr;
  double alpha = 1.0, beta = 0.0;
  double* slab = nullptr;
  const int* skip = nullptr;
  const float* X32 = nullptr;
  float* Y32 = nullptr;
  const int* f64flag = nullptr;
  const double* C2 = nullptr;
  const double* Z = nullptr;
  double* slab2 = nullptr;
  int mode = 0;
  int* grid_out = nullptr;  // rowgram_ex with grid <= 0: the grid it chose (per-CU occupancy)
  bool tri = false;         // C (and C2) upper triangular: all-zero MFMA blocks skipped (exact)
};
bool rowgram_ex(int64_t nrows, int b, const RowOpArgs& a, int grid, hipStream_t s);

// --- spmm.hip ----------------------------------------------------------------------------
// U = A * Qin  (+ epilogue U -= Qprev * Bt^T with Bt = B_i row-major b x b, if Qprev).
// variant: 0 auto, 1 global gather, 2 LDS window, 3 LDS band (MFMA), 4 band tiles (MFMA),
// 5 segmented gather (b in {16, 32}).
// ai_slab: if non-null and the band kernel runs with band_gram, it also forms the partials
// of A_i = Qin[own rows]^T U (b x b per workgroup) there; returns how many (0: not formed).
int spmm(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
         const double* Qprev, const double* Bi, int variant, hipStream_t s,
         double* ai_slab = nullptr);

bool spmm_seg_ok(const CsrDev& A, int b);
// column tiers (CsrDev::seg_tier): per row, the nonzeros of each tier (tier_of[col], uint8)
// counted into cnt[t * m + r], then copied in column order into the tier CSRs
void seg_tier_count(int64_t m, const int64_t* rowptr, const int32_t* col, const uint8_t* tier_of,
                    int ntiers, int32_t* cnt, hipStream_t s);
void seg_tier_fill(int64_t m, const int64_t* rowptr, const int32_t* col, const double* val,
                   const uint8_t* tier_of, int ntiers, int64_t* const* trp, int32_t* const* tcol,
                   double* const* tval, hipStream_t s);
// The same by a per-nonzero rule instead of tier_of[col] (TierRule: several ranks, the halo split
// into pulled and pushed products — rbl_api.cpp prepare_tiers): local row r (global row0 + r),
// column c: tier 0 if c is an own row; else tier 1 if c ranks above r — (deg[c], c) >
// (deg[r], r), deg indexed by global id — (the rank pulls Q_c); else tier 2 (the owner of c
// computes the product and pushes it).
struct TierRule {
  const int32_t* deg = nullptr;  // n entries (device); null: use tier_of
  int64_t row0 = 0, r0 = 0, r1 = 0;
};
void seg_tier_count_rule(int64_t m, const int64_t* rowptr, const int32_t* col, TierRule rule,
                         int32_t* cnt, hipStream_t s);
void seg_tier_fill_rule(int64_t m, const int64_t* rowptr, const int32_t* col, const double* val,
                        TierRule rule, int64_t* const* trp, int32_t* const* tcol,
                        double* const* tval, hipStream_t s);
// One tier as a plain CSR product: out[row] = sum_k val[k] Q[col[k] - col_off] (no epilogue),
// b in {16, 32} — the pushed partial rows of the halo split.
void spmm_seg_tier(const CsrDev::Tier& T, const double* Q, int64_t col_off, int b, double* out,
                   hipStream_t s);
// U[rows[i]] += sum_{k in [ptr[i], ptr[i+1])} recv[slot[k]] (slots in order: deterministic), b
// columns — the received pushed partials added to their rows.
void push_add(const int64_t* rows, const int64_t* ptr, const int64_t* slot, int64_t nrows,
              const double* recv, int b, double* U, hipStream_t s);
// spmm_panel.hip: column-panel CSR kernel for wide bands (b = 32, Q rows [q_lo, q_hi)); false
// if not applicable.  panel_width(): Q rows per panel.
bool spmm_panel(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
                const double* Qprev, const double* Bi, hipStream_t s);
int panel_width();
// the column-panel format (zeroed and filled on the device, stream-ordered): every row's count
// (cnt) and first record (st) in every panel of its block's window, and the records themselves
// regrouped panel-major within each block (pcol: column within the panel, pval: value); binfo
// on the device; ncnt entries of cnt / st, nnz records
int panel_format(const CsrDev& A, const int32_t* binfo, int R, int64_t nblk, uint16_t* cnt,
                 uint32_t* st, int64_t ncnt, uint8_t* pcol, double* pval, hipStream_t s);
// spmm_window.hip: persistent LDS-window kernel (b in {16,32}); false if not applicable.
bool spmm_window(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
                 const double* Qprev, const double* Bi, hipStream_t s);
int window_grid();              // workgroups for the window kernel (= CUs)
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) once per (device, kernel): thread-safe
// (in-process ranks launch from several threads) and per device (a process may drive several)
void ensure_lds_attr(const void* kernel, int bytes);
// spmm_band.hip: LDS-densified band tiles on fp64 MFMA (b in {16,32}); false if not applicable.
// ai_slab / ai_parts: see spmm().
bool spmm_band(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
               const double* Qprev, const double* Bi, hipStream_t s, double* ai_slab = nullptr,
               int* ai_parts = nullptr);
// spmm_bt.hip: band tiles in MFMA operand order streamed to VGPRs (b = 32, H in {32, 64});
// false if not applicable.
// Q32 / Qprev32 (optional, the fp32 basis): read fp32 blocks instead of Qin / Qprev.
bool spmm_bt_locfix_ok(const CsrDev& A, int b);
int spmm_bt_halfwidth(const CsrDev& A);
void spmm_bt_locfix_edges(const CsrDev& A, double* Q, const double* Qprev, const double* C,
                          int64_t lo0, int64_t hi0, int64_t lo1, int64_t hi1, hipStream_t s);
void spmm_bt_locfix_rest(const CsrDev& A, double* Q, const double* Qprev, const double* C,
                         hipStream_t s);
bool spmm_bt(const CsrDev& A, const double* Qin, int64_t col_off, int b, double* U,
             const double* Qprev, const double* Bi, hipStream_t s, double* ai_slab = nullptr,
             int* ai_parts = nullptr, const float* Q32 = nullptr, const float* Qprev32 = nullptr);
// band-tile format of the local CSR: tiles in consumption order (slot (round * grid + wg) * 4
// + wave), zero-filled `out` of bt_tile_slots(ntiles, tiles_per_wg) * NG * 256 doubles
// half tiles from the whole ones when the tiles are symmetric bit for bit (0; -1: not
// symmetric, nothing allocated; > 0: HIP error)
int bt_half(const double* full, int64_t ntiles, int64_t tpw, int NG, double** half,
            double** edge, hipStream_t s);
int64_t bt_tile_slots(int64_t ntiles, int64_t tiles_per_wg);
void bt_fill(const CsrDev& A, int H, int NG, double* out, hipStream_t s);
// packed band tiles from the dense ones (NG in {5, 9}): header words per tile slot, and the
// packed values (allocated here, *val_out; *nval_out values); returns 0 or a hipError_t
constexpr int bt_pack_words(int NG) { return (4 * NG + (2 * NG + 4) / 4 + 2) & ~1; }
int bt_pack(const double* dense, int64_t nslots, int NG, uint64_t* hdr, double** val_out,
            int64_t* nval_out, hipStream_t s);
constexpr int kWindowTileRows = 16;
// Band kernel geometry (host checks in rbl_api.cpp): a tile's band [c16, cmax] with
// c16 = cmin & ~15 spans <= kBandMaxK columns; the Q ring holds kBandRing rows; per tile a
// producer pass stores ring rows in whole sets of 512 / b (one element per producer thread).
constexpr int kBandMaxK = 176;
constexpr int kBandLd = 196;
constexpr int kBandRing = 256;
// positions of every nonzero in its tile's dense band (CsrDev::band_pos), from tile_info
void band_positions(const CsrDev& A, uint16_t* pos, hipStream_t s);

// --- tsmm.hip ----------------------------------------------------------------------------
// Partial Gram:  slab[s][a][c] = sum over rows of split s of W[r][a] * X[r][c]
//   W: run of nW panels (a in [0, nW*w)), X: panels (c in [0, X.count*X.w)).
// Returns the number of splits used; slab must hold splits * (nW*w) * (X.count*X.w).
int gram_splits(int64_t nrows, int nW, int w, int xcols);
void gram_partial(int64_t nrows, const PanelRun& W, const Panels& X, double* slab, int splits,
                  const int* skip, hipStream_t s);
// out[e] = sum_s slab[s][e], e < len.
void reduce_slab(const double* slab, int splits, int64_t len, double* out, const int* skip,
                 hipStream_t s);
// The same for tens of thousands of splits: a two-level sum whose first level writes
// reduce_scratch_splits(splits) x len doubles right after the partials (reserve them).
int reduce_scratch_splits(int splits);
void reduce_slab_many(double* slab, int splits, int64_t len, double* out, hipStream_t s);
// Y = beta*Y + alpha * X * C, X a run of panels (k = nX*X.w), C row-major k x (Y.count*Y.w)
// with leading dimension ldc.  Y may alias X's panels row-for-row (in-place apply).
void tsmm(int64_t nrows, const PanelRun& X, const double* C, int ldc, const Panels& Y,
          double alpha, double beta, const int* skip, hipStream_t s, double* xslab = nullptr,
          int* xgrid = nullptr);

// --- reorth.hip: v_mfma_f64_4x4x4f64 fast paths (panel widths 16 / 32), selected by
// gram_splits / gram_partial / tsmm above when applicable.
bool gram44_ok(int64_t nrows, int nW, int w, int xcount, int xw);
int gram44_splits(int64_t nrows, int nW, int w = 32);
void gram44_partial(int64_t nrows, const PanelRun& W, const Panels& X, double* slab, int splits,
                    const int* skip, hipStream_t s);
bool tsmm44_ok(int xw, int ky, int yw);
// Y = beta Y + alpha X C with X fp32 panels (X.base32), widened to fp64 as loaded: the Ritz
// projection over the fp32 basis in one pass (fp64 S and V).  Same shape limits as tsmm44.
void tsmm44_f32x(int64_t nrows, const PanelRun& X, const double* C, int ldc, const Panels& Y,
                 double alpha, double beta, hipStream_t s);
// xslab (optional, Y = [Q_i, Q_{i-1}] of width w = 16 or 32 on the fast path): also the
// partials of Q_{i-1}^T Q_i, *xgrid = tsmm44_xg_grid(nrows) blocks of w x w in xslab (one per
// 128-row tile; reduce_slab over *xgrid); *xgrid = 0 when this form does not apply.
int tsmm44_xg_grid(int64_t nrows);
void tsmm44(int64_t nrows, const PanelRun& X, const double* C, int ldc, const Panels& Y,
            double alpha, double beta, const int* skip, hipStream_t s, double* xslab = nullptr,
            int* xgrid = nullptr);

// --- reorth32.hip: the fp32 Krylov basis (mixed precision, b in {16, 32}) ---------------
// Gram partials slab[s][a][c] = sum over split s of W[r][a] X[r][c] (W: nW fp32 panels of
// width w at Wb + j*wstride, X: xcount fp32 panels of width w), fp32 MFMA per split.
int gram32_splits(int64_t nrows);
void gram32_partial(int64_t nrows, const float* Wb, int64_t wstride, int nW, int w, const float* X0,
                    const float* X1, int xcount, double* slab, int splits, hipStream_t s);
// Y = beta Y + alpha X C: X nX fp32 panels (k = nX*w), C fp64 row-major (rounded to f32),
// Y ycount fp32 panels of width w (Y may alias X's panels row-for-row).
void tsmm32(int64_t nrows, const float* Xb, int64_t xstride, int nX, int w, const double* C, int ldc,
            float* Y0, float* Y1, int ycount, float alpha, float beta, hipStream_t s);
void cvt_f32_to_f64(const float* src, double* dst, int64_t n, hipStream_t s);
void cvt_f64_to_f32(const double* src, float* dst, int64_t n, hipStream_t s);

// --- smallmat.hip ------------------------------------------------------------------------
// Cholesky step of (shifted) CholQR on the b x b Gram G (row-major, symmetric):
//   mode 0: first pass — try unshifted; on breakdown or estimated cond > 3e7 use the
//           Fukaya shift and set need3[0] = 1, need3[1] = 0 (so a third pass runs;
//           need3[1] is the `skip` word of the third pass' kernels);
//   mode 1: later pass — unshifted (falls back to shift if it still breaks).
// Writes R (upper), Rinv, and Rtot = R * Rtot_prev (first pass: Rtot = R).
// If *skip != 0 the kernel does nothing (used for the conditional third pass).
// scratch: 2 b^2 doubles (used only for b > 64: the factor and R^-1 do not fit in LDS there)
void chol_step(const double* G, int b, int64_t nglobal, int mode, double* R, double* Rinv,
               double* Rtot, int* need3, int* status, const int* skip, hipStream_t s,
               double* scratch);
// dst = src (len doubles): B_i stashed for the next step's epilogue, and the out-of-place
// CholQR applies at b > 64; nothing when *skip != 0.
void copy_small(const double* src, double* dst, int64_t len, hipStream_t s, const int* skip = nullptr);
// C = C Rinv (b x b, Rinv upper triangular) unless *skip (k_cloc_rinv)
void cloc_rinv(double* C, const double* Rinv, int b, const int* skip, hipStream_t s);
// dst = src^T (b x b row-major).
void transpose_small(const double* src, double* dst, int b, hipStream_t s);
// stash = [A_i (b x b) | R_tot (b x b) | 4 int flags], Bprev = R_tot, flags cleared (k_stash)
void stash_step(const double* Ai, const double* Rtot, double* Bprev, int* flags, double* stash,
                int b, hipStream_t s);

// --- gen_rmat.hip (R-MAT generator) -------------------------------------
struct RmatParams {
  int64_t n = 0;
  int scale = 0;
  int64_t edges = 0;
  double a = 0.57, b = 0.19, c = 0.19;
  uint64_t seed = 0;
  // RBL_OPT_RELABEL: the matrix is P A P^T, vertex v stored as row / column perm(v) (a seeded
  // Feistel bijection, make_scatter(n, seed ^ kRelabelK)); values and the planted diagonal
  // stay those of the original ids, so the spectrum is A's
  bool relabel = false;
  Scatter perm;
};
constexpr uint64_t kRelabelK = 0x52454C4142454C31ull;  // "RELABEL1"
// deg[r] += 1 per kept draw endpoint (duplicates counted; zero-filled deg of n int32)
void rmat_degree(const RmatParams& p, int32_t* deg, hipStream_t s);
// local CSR of rows [r0, r1): rowptr_dev (m+1, caller-allocated), col/val allocated here (with
// kCsrPad zero entries); max_keys >= the own rows' kept draw endpoints.  0 or a negative status.
int rmat_local_csr(const RmatParams& p, int64_t r0, int64_t r1, int64_t max_keys, int nplant,
                   const double* plant_dev, int64_t* rowptr_dev, int32_t** col_dev,
                   double** val_dev, int64_t* nnz_out, hipStream_t s);
// per-rank column footprint of a local CSR: lo[q] = min, hi[q] = max + 1 (atomics; lo/hi
// initialised to ~0 / 0), bounds_dev = the P+1 row boundaries
void col_footprint(const int32_t* col, int64_t nnz, const int64_t* bounds_dev, int P,
                   unsigned long long* lo, unsigned long long* hi, hipStream_t s);

// --- gen.hip ---------------------------------------------------------------------------
// Hash-window matrix rows [r0,r1): counts per row, then fill given rowptr (0-based, local).
// circuit-like matrix (gen.hip; oracle/matgen.py circuit_like_csr): rows [r0, r1) of the
// scattered index space, counts then CSR fill (columns sorted)
void circ_count(int64_t n, int64_t width, double p, uint64_t seed, int64_t r0, int64_t r1,
                int32_t* counts, hipStream_t s);
void circ_fill(int64_t n, int64_t width, double p, uint64_t seed, int64_t r0, int64_t r1,
               const int64_t* rowptr, int nplant, const double* plant_dev, int32_t* col,
               double* val, hipStream_t s);
// indexed halo (several ranks, unbanded A): out[i] = Q[idx[i]] (rows of b doubles); mark[c] = 1
// for every column c outside [r0, r1); col[k] = map[col[k]]
void gather_rows(const double* Q, const int32_t* idx, int64_t nrows, int b, double* out,
                 hipStream_t s);
void mark_cols(const int32_t* col, int64_t nnz, int64_t r0, int64_t r1, uint8_t* mark,
               hipStream_t s);
void remap_cols(int32_t* col, int64_t nnz, const int32_t* map, hipStream_t s);
void hw_count(int64_t n, int64_t W, double p, uint64_t seed, int64_t r0, int64_t r1,
              int32_t* counts, hipStream_t s);
void hw_fill(int64_t n, int64_t W, double p, uint64_t seed, int64_t r0, int64_t r1,
             const int64_t* rowptr, int nplant, const double* plant_dev, int32_t* col,
             double* val, hipStream_t s);
// N(0,1) block, row-major n_local x b, global row offset r0, counter-based from seed.
// N(0,1) start block of global rows r0.. (row r drawn from its id; with `perm` (the relabel of
// the matrix, RBL_OPT_RELABEL) from its original id perm^-1(r), so a relabelled run starts
// from the same block as the plain one, its rows permuted)
void randn_block(double* Q, int64_t nrows, int b, int64_t r0, uint64_t seed, hipStream_t s,
                 const Scatter* perm = nullptr);
// Per-tile column range of the CSR (tile = `tile_rows` rows), for the LDS-window SpMM.
void tile_col_range(const CsrDev& A, int tile_rows, int64_t* cmin, int64_t* cmax, hipStream_t s);
// column-major (ld = nrows) <-> row-major (ld = w) transposes for the boundary
void colmajor_to_rowmajor(const double* src, int64_t nrows, int w, double* dst, hipStream_t s);
void rowmajor_to_colmajor(const double* src, int64_t nrows, int w, double* dst, hipStream_t s);

}  // namespace rbl
