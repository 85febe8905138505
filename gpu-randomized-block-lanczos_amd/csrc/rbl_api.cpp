// rbl_api.cpp — the C-ABI of librbl_hip.so (include/rbl_hip.h).
//
// Host orchestration of one block Lanczos step on one GPU (or one rank of a row-partitioned
// job).  Mirrors the device part of Julia/RBL_gpu.jl:134-203; the CPU part (T_j band,
// dsbev, sort, convergence — Julia/common.jl) stays with the caller.
//
// HBM plan: A (CSR, int64 rowptr / int32 col / fp64 val), the WHOLE Krylov basis
// (max_blocks+1 slots of n_local x b, row-major), U, one scratch block, the Gram slab and
// b x b scalars.  Nothing but b x b blocks crosses PCIe per step.
#include <hip/hip_runtime.h>
#include <rocprofiler-sdk-roctx/roctx.h>

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/rbl_hip.h"
#include "comm.hpp"
#include "kernels.hpp"

using namespace rbl;

struct rbl_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  int nranks = 1, rank = 0;
  Comm* comm = nullptr;  // RCCL or in-process transport (comm.hpp); null for one rank
  std::string err;

  // matrix (local rows [r0,r1) of an n x n symmetric matrix)
  int64_t n = 0, r0 = 0, r1 = 0, nloc = 0, nnz = 0;
  int64_t* d_rowptr = nullptr;
  int32_t* d_col = nullptr;
  double* d_val = nullptr;
  int64_t* d_tcmin = nullptr;
  int64_t* d_tcmax = nullptr;
  int64_t* d_tinfo = nullptr;
  // column-panel SpMM (spmm_panel.hip): per 256-row block its first and last 256-row Q panel
  int32_t* d_panel_blk = nullptr;
  uint16_t* d_panel_cnt = nullptr;  // per block, panel and row: the row's entries in the panel
  uint32_t* d_panel_st = nullptr;   // ... and their first record (from the block's base)
  uint8_t* d_panel_col = nullptr;   // the records panel-major within a block: column in the panel
  double* d_panel_val = nullptr;    //   and value
  int64_t panel_nblk = 0;
  int panel_rpg = 4;        // rows per 16-lane group: blocks of 64 panel_rpg rows
  int panel_ch = 48;        // records per row and chunk load
  bool panel_auto = false;  // chosen by default: every staged Q row used >= 4 times on average
  int64_t panel_span = 0;   // the widest block window, Q rows
  uint16_t* d_bpos = nullptr;  // band kernel: per-nonzero dense-tile positions
  double* d_bt = nullptr;      // band-tile kernel: the CSR in MFMA-ordered 16-row band tiles
  int bt_ng = 0;               // its band groups (0: not applicable)
  uint64_t* d_btp_hdr = nullptr;  // the band tiles packed (zeros dropped; replaces d_bt)
  double* d_bth = nullptr;        // half band tiles (A symmetric; replaces d_bt), and the
  double* d_bte = nullptr;        //   first (NG-1)/2 local tiles whole
  double* d_btp_val = nullptr;
  double* d_zrow = nullptr;    // 32 zeros: band rows the halo does not hold
  // segmented-gather task table (spmm.hip variant 5; CsrDev::seg_*)
  int64_t seg_ntasks = 0, seg_nlong = 0;
  int64_t* d_seg_trow = nullptr;
  int32_t* d_seg_tinfo = nullptr;
  int64_t* d_seg_slot_k0 = nullptr;
  int64_t* d_seg_lrow = nullptr;
  int64_t* d_seg_lslot = nullptr;
  double* d_seg_scratch = nullptr;
  // column tiers of the segmented gather (RBL_SEG_TIERS, one rank; CsrDev::seg_tier): each a
  // CSR of the same rows holding the nonzeros of one column-degree tier, with its task table
  struct SegTierBuf {
    int64_t* rowptr = nullptr;
    int32_t* col = nullptr;
    double* val = nullptr;
    int64_t ntasks = 0, nlong = 0;
    int64_t* trow = nullptr;
    int32_t* tinfo = nullptr;
    int64_t* slot_k0 = nullptr;
    int64_t* lrow = nullptr;
    int64_t* lslot = nullptr;
    double* scratch = nullptr;
  };
  int seg_ntiers = 0;
  SegTierBuf seg_tier[3];
  bool seg_split = false;             // several ranks: tiers = own / halo columns
  // indexed halo (with seg_split): the halo tier's columns renumbered to ghost slots
  // [0, n_ghost) in d_qext, grouped by owning rank; each step every rank packs the rows its
  // peers asked for (d_send_idx, local row ids grouped by peer) and sends only those
  bool ghost = false;
  int64_t n_ghost = 0, n_send = 0;
  std::vector<int64_t> ghost_cnt, ghost_off, send_cnt, send_off;
  int32_t* d_send_idx = nullptr;
  double* d_sendbuf = nullptr;        // n_send x b, per run
  const double* ghost_local = nullptr;  // the block the last exchange sent from
  bool ghost_active = false;          // the last exchange was the indexed one (use_ghost)
  bool halo_overlap = true;           // RBL_OPT_HALO_OVERLAP
  // push/pull split of the indexed halo (RBL_OPT_HALO_PUSH): of every off-rank product
  // A[r,c] Q[c] the rank holding the higher-ranked endpoint ((degree, id) order) does the work —
  // it pulls Q[c] when c ranks higher (tier 1: the ghost slots), and when r ranks higher the
  // owner of c computes A[c,r] Q[c] from its own rows and pushes the partial row r (the push
  // tier, rows = ghost slots of that owner, columns = its own rows); received partials are
  // added to U in peer order (d_ps_*)
  int halo_push_opt = 2;              // 0 off, 1 on, 2 on when it moves fewer rows (default)
  bool push = false;
  SegTierBuf push_tier;
  int64_t push_rows = 0;              // = n_ghost (rows of the push tier)
  double* d_pushbuf = nullptr;        // n_ghost x b: pushed partial rows (per run)
  double* d_precv = nullptr;          // n_send x b: partial rows received for own rows (per run)
  int64_t* d_ps_rows = nullptr;       // own rows that receive partials, ascending
  int64_t* d_ps_ptr = nullptr;        //   their slots in d_precv (peer order)
  int64_t* d_ps_slot = nullptr;
  int64_t n_ps_rows = 0;
  size_t push_cap = 0;                // capacity (doubles) of d_pushbuf / d_precv
  int64_t push_pred_rows = 0, pull_pred_rows = 0;  // rows per SpMM, summed over ranks (setup)
  hipEvent_t ev_push_ready = nullptr, ev_push_done = nullptr;
  hipStream_t hstream = nullptr;      // the overlapped halo exchange
  hipEvent_t ev_qready = nullptr, ev_halo = nullptr;
  // dense A (RBL_gpu(A::Matrix{Float64})): local rows in 32-column row-major panels
  // (panel p = columns [32p, 32p+32), zero past n), multiplied by tsmm44 against d_qfull
  // (all n rows of Q, zero-padded to 32 * dense_panels rows, b <= 64 columns)
  bool dense = false;
  double* d_dense = nullptr;
  int64_t dense_panels = 0;
  double* d_qfull = nullptr;
  int qfull_cols = 0;         // columns d_qfull was sized for
  int64_t ntiles = 0, tiles_per_wg = 0;
  bool window_ok16 = false, window_ok32 = false;
  bool band_ok16 = false, band_ok32 = false;
  bool band_gram = false;                 // band kernel may form A_i (tile rows ring-resident)
  bool band_pair = false;                 // band kernel may stage row pairs with one load set
  std::vector<int64_t> bounds;            // nranks+1
  std::vector<int64_t> need_lo, need_hi;  // rows I need from rank q
  std::vector<int64_t> give_lo, give_hi;  // rows rank q needs from me
  int64_t ext_lo = 0, ext_hi = 0;         // global rows held in d_qext
  bool split_halo = true;                 // RBL_OPT_SPLIT_HALO
  bool keep_csr = true;                   // RBL_OPT_KEEP_CSR
  int relabel_opt = 0;                    // RBL_OPT_RELABEL (applies to the next generator call)
  bool relabeled = false;                 // the matrix held is P A P^T (rmat generator)
  Scatter relabel_perm;                   //   with this P: vertex v at row perm(v)
  bool csr_dropped = false;               // values / column ids released (band tiles only)

  // Krylov run
  int b = 0, max_blocks = 0, nblocks = 0;
  double* d_basis = nullptr;  // (max_blocks+1) slots (fp64 basis)
  int64_t slot = 0;           // nloc * b
  // fp32 basis (mixed precision, RBL_gpu.jl with FLOAT = Float32): slots in d_basis32, the
  // current and previous block widened to fp64 in d_Qi64 / d_Qm64 for A Q, 3-term and QR
  int basis_bits = 64;
  // host spill (RBL_OPT_DEVICE_BLOCKS): blocks j < resident live in d_basis slot j; blocks
  // j >= resident in working slot resident + (j & 1) while among the two newest, and in
  // pinned host slot j - resident once final (copied during step j + 2)
  int dev_blocks_opt = 0;
  bool auto_planned = false;  // the current basis plan came from RBL_OPT_DEVICE_BLOCKS = -1
  int resident = INT32_MAX;
  // pinned host slots of the spilled blocks (block j at h_spill[j - resident]), pinned when
  // the block is first written out: host memory grows with the blocks a run really spills
  std::vector<void*> h_spill;
  double* d_stage = nullptr;          // one n_local x b staging block for spilled blocks
  hipStream_t cstream = nullptr;      // D2H copies of finished spilled blocks
  hipEvent_t ev_fin = nullptr, ev_d2h[2] = {nullptr, nullptr};
  // rbl_step_async: step i's stash (A_i, R_tot, flags) has landed when step_ev[i] completes, so
  // rbl_fetch waits for the steps it returns, not for steps enqueued after them
  std::vector<hipEvent_t> step_ev;
  bool d2h_pending[2] = {false, false};
  float* d_basis32 = nullptr;
  float* d_stage32 = nullptr;
  double* d_Qi64 = nullptr;
  double* d_Qm64 = nullptr;
  double* d_U = nullptr;
  double* d_T = nullptr;      // scratch n_local x max(b,k)
  int64_t T_cols = 0;
  double* d_qext = nullptr;   // halo-extended Q_i (multi-rank)
  size_t qext_cap = 0;        // its capacity in doubles (grown by ensure_qext)
  double* d_slab = nullptr;
  size_t slab_elems = 0;
  double* d_C = nullptr;      // Gram result (<= (max_blocks)*b x 2b)
  size_t C_elems = 0;
  double* d_small = nullptr;  // R, Rinv, Rtot, Bprev, Ai, G (b x b each)
  int* d_flags = nullptr;     // [need3, skip3, status0, status1]
  double* h_pin = nullptr;    // pinned staging: Ai, Rtot (2 b x b)
  void* h_d2h[2] = {nullptr, nullptr};  // pinned slots of the staged D2H (d2h_staged)
  hipEvent_t ev_d2h_slot[2] = {nullptr, nullptr};
  hipStream_t rstream = nullptr;      // the Ritz row pieces (ritz_pipelined)
  hipEvent_t ev_ritz[9] = {};         // S uploaded, then each row piece finished on rstream
  double* h_hist = nullptr;   // rbl_step_async stash: per step i, Ai and Rtot (2 b x b) and the
                              //   step's 4 flags (2 doubles' room): stash_rec(b) doubles each
  double* d_stash = nullptr;  // the device side of one such record (k_stash; RBL_STASH_COPY=1)
  // k_stash writes the record straight into h_pin / h_hist (coherent pinned memory, these are
  // their device addresses) instead of a device record plus a D2H copy, which the SDMA engine
  // ran ~60-80 us after the kernel, on the step's critical path
  bool stash_direct = true;
  double* dv_pin = nullptr;
  double* dv_hist = nullptr;
  bool flags_clean = false;   // d_flags already zero (the last step's k_stash cleared them)
  int fetched = 1;            // steps < fetched have been returned by rbl_fetch
  bool have_bprev = false;
  // locked Ritz vectors of the restarted variants (restarted.jl: Qlock / Qlock_gpu), fp64,
  // vector j at d_lock + j * nloc (a width-1 panel)
  double* d_lock = nullptr;
  int nlock = 0, lock_cap = 0;

  // options
  int timers = 0;  // RBL_OPT_TIMERS: 0 off, 1 every stage, 2 the SpMM and partial-reorth stages
  int reorth_order = 0;
  int spmm_variant = 0;
  int fuse = 7;               // RBL_OPT_FUSE
  // the local-reorth coefficient Q_{i-1}^T Q_i of step cloc_step (S_CLOC), formed by the QR of
  // step cloc_step - 1 or by the last partial-reorth update of step cloc_step; 0: none
  int cloc_step = 0;
  bool cloc_final = false;    // formed after this step's reorth (valid whatever its flags)
  std::vector<int> step_flags;  // part_reorth flags per step (the fusion's schedule guess)
  double stage_ms[RBL_NUM_STAGES] = {0};
  // collectives issued by this rank since the last reset (rbl_comm_stats): all-reduce calls and
  // bytes, grouped halo exchanges and the bytes sent / received in them
  int64_t comm_stats[RBL_COMM_NSTATS] = {0};
  // time spent in this rank's collectives since the last rbl_comm_stats reset
  // (RBL_COMM_*_HOST_NS / *_DEV_NS): host wall time inside the transport call, and the
  // hipEvent span of the call on its stream (recorded while RBL_OPT_TIMERS is 1)
  int64_t comm_host_ns[2] = {0, 0};  // [0] all-reduces, [1] halo exchanges
  double comm_dev_ms[2] = {0.0, 0.0};
  // which code path each step took (rbl_path_stats): counted on the host as the work is issued,
  // so a test can assert the path itself instead of timing it
  int64_t path_stats[RBL_PATH_NSTATS] = {0};
  // parent: the stage whose span encloses this one on the same stream (a collective inside
  // "3-term" / "qr" / "part reorth"), whose time excludes it; -1 none
  struct Mark { int stage; hipEvent_t a, b; int parent = -1; };
  std::vector<Mark> marks;
  struct OpenStage { int stage; hipStream_t st; };
  std::vector<OpenStage> open_stages;  // StageScopes alive now, innermost last
  std::vector<hipEvent_t> ev_pool;
  size_t ev_used = 0;
};

namespace {

const char* kStageNames[RBL_NUM_STAGES] = {"AQ", "3-term", "qr", "part reorth", "loc reorth",
                                           "Ritz vectors", "comm", "spill wait"};

int fail(rbl_ctx* c, int code, const std::string& msg) {
  if (c) c->err = msg;
  return code;
}

// device allocation released on every return path
struct DevBuf {
  void* p = nullptr;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  double* d() const { return static_cast<double*>(p); }
};

#define HIPC(expr)                                                                    \
  do {                                                                                \
    hipError_t _e = (expr);                                                           \
    if (_e != hipSuccess)                                                             \
      return fail(ctx, _e == hipErrorOutOfMemory ? RBL_ERR_OOM : RBL_ERR_HIP,          \
                  std::string(#expr) + ": " + hipGetErrorString(_e));                 \
  } while (0)
#define COMMC(expr)               \
  do {                            \
    int _s = (expr);              \
    if (_s < 0) return _s;        \
  } while (0)
#define CHK(expr)             \
  do {                        \
    int _s = (expr);          \
    if (_s < 0) return _s;    \
  } while (0)

// device location of fp64 block j: resident slot, or (spilled region) its working slot —
// valid only while j is one of the two newest blocks
double* slotp(rbl_ctx* ctx, int j) {
  const int s = j < ctx->resident ? j : ctx->resident + (j & 1);
  return ctx->d_basis + (int64_t)s * ctx->slot;
}
bool spilled(const rbl_ctx* ctx) { return ctx->resident != INT32_MAX; }
// fp64 block j on the device: in place when resident or among the newest two of `nblocks`,
// else copied from pinned host memory into the staging block (on the compute stream)
const double* block_dev(rbl_ctx* ctx, int j, int nblocks, int* st) {
  *st = 0;
  if (j < ctx->resident || j >= nblocks - 2) return slotp(ctx, j);
  const hipError_t e = hipMemcpyAsync(ctx->d_stage, ctx->h_spill[j - ctx->resident],
                                      ctx->slot * sizeof(double), hipMemcpyHostToDevice, ctx->stream);
  if (e != hipSuccess) *st = RBL_ERR_HIP;
  return ctx->d_stage;
}
// fp32 basis: the same slot plan as slotp / block_dev
// pin the host slot of spilled block j on first use (non-coherent pages: the DMA engines
// stream them at PCIe rate both ways)
int spill_slot(rbl_ctx* ctx, int j, size_t elem) {
  void*& h = ctx->h_spill[j - ctx->resident];
  if (!h) {
    const hipError_t e = hipHostMalloc(&h, (size_t)ctx->slot * elem, hipHostMallocNonCoherent);
    if (e != hipSuccess) {
      h = nullptr;
      return fail(ctx, e == hipErrorOutOfMemory ? RBL_ERR_OOM : RBL_ERR_HIP,
                  std::string("host spill: hipHostMalloc: ") + hipGetErrorString(e));
    }
  }
  return RBL_OK;
}
float* slotp32(rbl_ctx* ctx, int j) {
  const int s = j < ctx->resident ? j : ctx->resident + (j & 1);
  return ctx->d_basis32 + (int64_t)s * ctx->slot;
}
const float* block_dev32(rbl_ctx* ctx, int j, int nblocks, int* st) {
  *st = 0;
  if (j < ctx->resident || j >= nblocks - 2) return slotp32(ctx, j);
  const hipError_t e = hipMemcpyAsync(ctx->d_stage32, ctx->h_spill[j - ctx->resident],
                                      ctx->slot * sizeof(float), hipMemcpyHostToDevice, ctx->stream);
  if (e != hipSuccess) *st = RBL_ERR_HIP;
  return ctx->d_stage32;
}

CsrDev csr(rbl_ctx* ctx) {
  CsrDev A;
  A.nrows = ctx->nloc;
  A.nnz = ctx->nnz;
  A.rowptr = ctx->d_rowptr;
  A.col = ctx->d_col;
  A.val = ctx->d_val;
  A.tile_cmin = ctx->d_tcmin;
  A.tile_cmax = ctx->d_tcmax;
  A.tile_info = ctx->d_tinfo;
  // (the indexed halo's buffer holds ghost slots, not a row range: the panels need the range)
  A.panel_blk = ctx->ghost ? nullptr : ctx->d_panel_blk;
  A.panel_nblk = ctx->ghost ? 0 : ctx->panel_nblk;
  A.panel_auto = ctx->panel_auto;
  A.panel_cnt = ctx->d_panel_cnt;
  A.panel_st = ctx->d_panel_st;
  A.panel_col = ctx->d_panel_col;
  A.panel_val = ctx->d_panel_val;
  A.panel_rpg = ctx->panel_rpg;
  A.panel_ch = ctx->panel_ch;
  A.ntiles = ctx->ntiles;
  A.tiles_per_wg = ctx->tiles_per_wg;
  A.window_ok16 = ctx->window_ok16;
  A.window_ok32 = ctx->window_ok32;
  A.band_ok16 = ctx->band_ok16;
  A.band_ok32 = ctx->band_ok32;
  A.band_gram = ctx->band_gram;
  A.band_pair = ctx->band_pair;
  A.row0 = ctx->r0;
  A.band_pos = ctx->d_bpos;
  A.bt = ctx->d_bt;
  A.bth = ctx->d_bth;
  A.bte = ctx->d_bte;
  A.bt_ng = ctx->bt_ng;
  A.btp_hdr = ctx->d_btp_hdr;
  A.btp_val = ctx->d_btp_val;
  A.bt_tiles_per_wg = ctx->tiles_per_wg;
  A.q_lo = ctx->nranks > 1 ? ctx->ext_lo : ctx->r0;
  A.q_hi = ctx->nranks > 1 ? ctx->ext_hi : ctx->r0 + ctx->nloc;
  A.zrow = ctx->d_zrow;
  A.seg_ntasks = ctx->seg_ntasks;
  A.seg_trow = ctx->d_seg_trow;
  A.seg_tinfo = ctx->d_seg_tinfo;
  A.seg_slot_k0 = ctx->d_seg_slot_k0;
  A.seg_nlong = ctx->seg_nlong;
  A.seg_lrow = ctx->d_seg_lrow;
  A.seg_lslot = ctx->d_seg_lslot;
  A.seg_scratch = ctx->d_seg_scratch;
  A.seg_ntiers = ctx->seg_ntiers;
  A.seg_split = ctx->seg_split;
  for (int t = 0; t < ctx->seg_ntiers; ++t) {
    const auto& T = ctx->seg_tier[t];
    auto& D = A.seg_tier[t];
    D.rowptr = T.rowptr;
    D.col = T.col;
    D.val = T.val;
    D.ntasks = T.ntasks;
    D.nlong = T.nlong;
    D.trow = T.trow;
    D.tinfo = T.tinfo;
    D.slot_k0 = T.slot_k0;
    D.lrow = T.lrow;
    D.lslot = T.lslot;
    D.scratch = T.scratch;
  }
  return A;
}

// Task table of the segmented gather (spmm.hip variant 5): short rows packed into tasks of
// <= kSegPack nonzeros and <= 64 rows, rows over kSegLen nonzeros cut into segments.
int build_seg(rbl_ctx* ctx, const std::vector<int64_t>& rp, rbl_ctx::SegTierBuf& out) {
  const int64_t m = (int64_t)rp.size() - 1;
  if (m <= 0) return RBL_OK;
  std::vector<int64_t> trow, slot_k0, lrow, lslot;
  std::vector<int32_t> tinfo;
  int64_t cur_r0 = 0, cur_nnz = 0;
  int cur_rows = 0;
  auto flush = [&]() {
    if (cur_rows) {
      trow.push_back(cur_r0);
      tinfo.push_back(cur_rows);
    }
    cur_rows = 0;
    cur_nnz = 0;
  };
  for (int64_t r = 0; r < m; ++r) {
    const int64_t d = rp[r + 1] - rp[r];
    if (d > kSegLen) {
      flush();
      lrow.push_back(r);
      lslot.push_back((int64_t)slot_k0.size());
      for (int64_t k = rp[r]; k < rp[r + 1]; k += kSegLen) {
        trow.push_back(r);
        tinfo.push_back(-(int32_t)(slot_k0.size() + 1));
        slot_k0.push_back(k);
      }
      continue;
    }
    if (cur_rows && (cur_nnz + d > kSegPack || cur_rows == 64)) flush();
    if (!cur_rows) cur_r0 = r;
    ++cur_rows;
    cur_nnz += d;
  }
  flush();
  lslot.push_back((int64_t)slot_k0.size());
  slot_k0.push_back(INT64_MAX);
  out.ntasks = (int64_t)trow.size();
  out.nlong = (int64_t)lrow.size();
  HIPC(hipMalloc(&out.trow, trow.size() * sizeof(int64_t)));
  HIPC(hipMalloc(&out.tinfo, tinfo.size() * sizeof(int32_t)));
  HIPC(hipMalloc(&out.slot_k0, slot_k0.size() * sizeof(int64_t)));
  HIPC(hipMalloc(&out.lslot, lslot.size() * sizeof(int64_t)));
  HIPC(hipMalloc(&out.lrow, std::max<size_t>(lrow.size(), 1) * sizeof(int64_t)));
  HIPC(hipMalloc(&out.scratch, std::max<size_t>(slot_k0.size() - 1, 1) * 32 * sizeof(double)));
  HIPC(hipMemcpy(out.trow, trow.data(), trow.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  HIPC(hipMemcpy(out.tinfo, tinfo.data(), tinfo.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  HIPC(hipMemcpy(out.slot_k0, slot_k0.data(), slot_k0.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  HIPC(hipMemcpy(out.lslot, lslot.data(), lslot.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  if (!lrow.empty())
    HIPC(hipMemcpy(out.lrow, lrow.data(), lrow.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  return RBL_OK;
}

void free_seg(rbl_ctx::SegTierBuf& T, bool with_csr) {
  if (with_csr) {
    hipFree(T.rowptr);
    hipFree(T.col);
    hipFree(T.val);
  }
  hipFree(T.trow);
  hipFree(T.tinfo);
  hipFree(T.slot_k0);
  hipFree(T.lrow);
  hipFree(T.lslot);
  hipFree(T.scratch);
  T = rbl_ctx::SegTierBuf();
}

// the column-panel format (spmm_panel.hip) and its choice
void free_panels(rbl_ctx* ctx) {
  hipFree(ctx->d_panel_blk); ctx->d_panel_blk = nullptr; ctx->panel_nblk = 0; ctx->panel_auto = false;
  ctx->panel_span = 0;
  hipFree(ctx->d_panel_cnt); ctx->d_panel_cnt = nullptr;
  hipFree(ctx->d_panel_st); ctx->d_panel_st = nullptr;
  hipFree(ctx->d_panel_col); ctx->d_panel_col = nullptr;
  hipFree(ctx->d_panel_val); ctx->d_panel_val = nullptr;
}

void free_tiers(rbl_ctx* ctx) {
  for (auto& T : ctx->seg_tier) free_seg(T, true);
  ctx->seg_ntiers = 0;
  ctx->seg_split = false;
  hipFree(ctx->d_send_idx); ctx->d_send_idx = nullptr;
  ctx->ghost = false;
  ctx->n_ghost = ctx->n_send = 0;
  free_seg(ctx->push_tier, true);
  ctx->push = false;
  ctx->push_rows = 0;
  hipFree(ctx->d_ps_rows); ctx->d_ps_rows = nullptr;
  hipFree(ctx->d_ps_ptr); ctx->d_ps_ptr = nullptr;
  hipFree(ctx->d_ps_slot); ctx->d_ps_slot = nullptr;
  ctx->n_ps_rows = 0;
}

int prepare_segments(rbl_ctx* ctx, const std::vector<int64_t>& rp) {
  if (ctx->nloc <= 0 || ctx->nnz <= 0) return RBL_OK;
  rbl_ctx::SegTierBuf T;
  const int st = build_seg(ctx, rp, T);
  ctx->seg_ntasks = T.ntasks;
  ctx->seg_nlong = T.nlong;
  ctx->d_seg_trow = T.trow;
  ctx->d_seg_tinfo = T.tinfo;
  ctx->d_seg_slot_k0 = T.slot_k0;
  ctx->d_seg_lrow = T.lrow;
  ctx->d_seg_lslot = T.lslot;
  ctx->d_seg_scratch = T.scratch;
  return st;
}

int build_tiers(rbl_ctx* ctx, const std::vector<uint8_t>& tier_of, int nt,
                const TierRule* rule = nullptr);

// nonzeros of tier t (its row pointer's last entry)
int64_t tier_nnz(rbl_ctx* ctx, int t) {
  int64_t v = 0;
  if (ctx->seg_tier[t].rowptr && ctx->nloc > 0)
    (void)hipMemcpy(&v, ctx->seg_tier[t].rowptr + ctx->nloc, sizeof(int64_t), hipMemcpyDeviceToHost);
  return v;
}

// Indexed halo: the columns this rank references outside its rows become ghost slots (sorted by
// global id, so grouped by owner); the ranks exchange how many rows, then which rows, each asks
// of each; *d_map (device, n int32) maps a ghost column to its slot (caller frees).
int build_ghosts(rbl_ctx* ctx, int32_t** d_map, const int32_t* cols, int64_t ncols) {
  const int P = ctx->nranks, me = ctx->rank;
  const int64_t n = ctx->n;
  uint8_t* d_mark = nullptr;
  HIPC(hipMalloc(&d_mark, std::max<int64_t>(n, 1)));
  HIPC(hipMemsetAsync(d_mark, 0, n, ctx->stream));
  mark_cols(cols, ncols, ctx->r0, ctx->r1, d_mark, ctx->stream);
  HIPC(hipGetLastError());
  std::vector<uint8_t> mark(n);
  HIPC(hipMemcpyAsync(mark.data(), d_mark, n, hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  hipFree(d_mark);
  std::vector<int32_t> map(n, 0);
  std::vector<int64_t> req;  // global ids of the ghost rows, ascending
  ctx->ghost_cnt.assign(P, 0);
  ctx->ghost_off.assign(P, 0);
  for (int q = 0; q < P; ++q) {
    ctx->ghost_off[q] = (int64_t)req.size();
    if (q == me) continue;
    for (int64_t c = ctx->bounds[q]; c < ctx->bounds[q + 1]; ++c)
      if (mark[c]) {
        map[c] = (int32_t)req.size();
        req.push_back(c);
      }
    ctx->ghost_cnt[q] = (int64_t)req.size() - ctx->ghost_off[q];
  }
  ctx->n_ghost = (int64_t)req.size();
  // what each peer asks of me: row `me` of the all-gathered count table, column by column
  std::vector<int64_t> all((size_t)P * P);
  COMMC(ctx->comm->allgather_host(ctx->ghost_cnt.data(), all.data(), P, ctx->stream, &ctx->err));
  ctx->send_cnt.assign(P, 0);
  ctx->send_off.assign(P, 0);
  int64_t ns = 0;
  for (int q = 0; q < P; ++q) {
    ctx->send_off[q] = ns;
    ctx->send_cnt[q] = q == me ? 0 : all[(size_t)q * P + me];
    ns += ctx->send_cnt[q];
  }
  ctx->n_send = ns;
  // the request lists themselves, int64 ids carried as 8-byte words by the halo transport
  DevBuf d_req, d_got;
  HIPC(hipMalloc(&d_req.p, std::max<int64_t>(ctx->n_ghost, 1) * sizeof(int64_t)));
  HIPC(hipMalloc(&d_got.p, std::max<int64_t>(ns, 1) * sizeof(int64_t)));
  if (ctx->n_ghost)
    HIPC(hipMemcpy(d_req.p, req.data(), ctx->n_ghost * sizeof(int64_t), hipMemcpyHostToDevice));
  std::vector<Comm::Xfer> x(P);
  for (int q = 0; q < P; ++q) {
    if (q == me) continue;
    x[q].send = d_req.d() + ctx->ghost_off[q];
    x[q].nsend = (size_t)ctx->ghost_cnt[q];
    x[q].recv = d_got.d() + ctx->send_off[q];
    x[q].nrecv = (size_t)ctx->send_cnt[q];
  }
  COMMC(ctx->comm->exchange(x, ctx->stream, &ctx->err));
  std::vector<int64_t> got(std::max<int64_t>(ns, 1));
  HIPC(hipMemcpyAsync(got.data(), d_got.p, ns * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  std::vector<int32_t> idx(std::max<int64_t>(ns, 1), 0);
  for (int64_t i = 0; i < ns; ++i) {
    const int64_t g = got[i] - ctx->r0;
    if (g < 0 || g >= ctx->nloc) return fail(ctx, RBL_ERR_INVALID, "indexed halo: a peer asked for a row I do not own");
    idx[i] = (int32_t)g;
  }
  HIPC(hipMalloc(&ctx->d_send_idx, std::max<int64_t>(ns, 1) * sizeof(int32_t)));
  if (ns) HIPC(hipMemcpy(ctx->d_send_idx, idx.data(), ns * sizeof(int32_t), hipMemcpyHostToDevice));
  HIPC(hipMalloc(d_map, std::max<int64_t>(n, 1) * sizeof(int32_t)));
  HIPC(hipMemcpy(*d_map, map.data(), n * sizeof(int32_t), hipMemcpyHostToDevice));
  return RBL_OK;
}

// Push/pull split of the indexed halo (several ranks, unbanded A).  Every off-rank product
// A[r,c] Q[c] is done by the rank of the endpoint that ranks higher by (row degree, smaller id):
// when c ranks higher the rank of r pulls Q[c] (tier 1, as in the pull-all halo), otherwise the
// rank of c — which holds A[c,r] = A[r,c] in its own rows — forms it from its own Q rows and
// pushes the partial row r (tier 2 is dropped: its products arrive pushed).  Hub rows (the
// high-degree rows of a power-law graph, referenced from every rank) then stay home and only
// their partials move, one row per (hub, rank) pair in each direction.  The push tier is tier
// 1 transposed (rows: the ghost slots, columns: own rows), so ghosts pulled = partials pushed.
// Returns 1 when set up, 0 when the pull-all halo is to be used — off (RBL_OPT_HALO_PUSH 0),
// predicted to move more rows (automatic: used when 2 x ghosts(tier 1) < 0.85 x ghosts(all),
// summed over ranks), or A not structurally symmetric by the per-pair entry counts — the
// same answer on every rank; < 0 on error.  Collective.
int prepare_push(rbl_ctx* ctx, const std::vector<int64_t>& rp) {
  const int P = ctx->nranks;
  const int64_t n = ctx->n, m = ctx->nloc;
  // global row degrees: every rank's slice (padded to the longest) all-gathered
  int64_t w = 1;
  for (int q = 0; q < P; ++q) w = std::max(w, ctx->bounds[q + 1] - ctx->bounds[q]);
  std::vector<int64_t> mine(w, 0), all((size_t)P * w);
  for (int64_t r = 0; r < m && r + 1 < (int64_t)rp.size(); ++r) mine[r] = rp[r + 1] - rp[r];
  COMMC(ctx->comm->allgather_host(mine.data(), all.data(), w, ctx->stream, &ctx->err));
  std::vector<int32_t> deg(std::max<int64_t>(n, 1), 0);
  for (int q = 0; q < P; ++q)
    for (int64_t i = 0; i < ctx->bounds[q + 1] - ctx->bounds[q]; ++i)
      deg[ctx->bounds[q] + i] = (int32_t)std::min<int64_t>(all[(size_t)q * w + i], INT32_MAX);
  std::vector<int64_t>().swap(all);
  DevBuf d_deg;
  HIPC(hipMalloc(&d_deg.p, deg.size() * sizeof(int32_t)));
  HIPC(hipMemcpy(d_deg.p, deg.data(), deg.size() * sizeof(int32_t), hipMemcpyHostToDevice));
  TierRule R;
  R.deg = static_cast<const int32_t*>(d_deg.p);
  R.row0 = ctx->r0;
  R.r0 = ctx->r0;
  R.r1 = ctx->r1;
  CHK(build_tiers(ctx, {}, 3, &R));
  // per peer: my tier-1 / tier-2 entries by the owner of their column, and the distinct
  // columns of tier 1 (the ghosts with the split) and of tiers 1 + 2 (without)
  const int64_t nz1 = m > 0 ? tier_nnz(ctx, 1) : 0, nz2 = m > 0 ? tier_nnz(ctx, 2) : 0;
  std::vector<int32_t> c1(std::max<int64_t>(nz1, 1)), c2(std::max<int64_t>(nz2, 1));
  // [tier-1 entries by owner | tier-2 by owner | d1 | d12 | tier-1 hash by owner | tier-2 hash |
  //  this rank's status]: a rank whose local part fails (a D2H copy) still takes part in the
  // all-gather with its error code, and every rank then fails together instead of leaving its
  // peers waiting in the collective
  std::vector<int64_t> vote(4 * P + 3, 0);
  auto owner = [&](int64_t c) {
    return (int)(std::upper_bound(ctx->bounds.begin(), ctx->bounds.end(), c) - ctx->bounds.begin()) - 1;
  };
  auto local_counts = [&]() -> int {
    if (nz1) HIPC(hipMemcpy(c1.data(), ctx->seg_tier[1].col, nz1 * sizeof(int32_t), hipMemcpyDeviceToHost));
    if (nz2) HIPC(hipMemcpy(c2.data(), ctx->seg_tier[2].col, nz2 * sizeof(int32_t), hipMemcpyDeviceToHost));
    std::vector<uint8_t> mark(std::max<int64_t>(n, 1), 0);
    for (int64_t k = 0; k < nz1; ++k) {
      ++vote[owner(c1[k])];
      if (!mark[c1[k]]) { mark[c1[k]] = 1; ++vote[2 * P]; }
    }
    for (int64_t k = 0; k < nz2; ++k) {
      ++vote[P + owner(c2[k])];
      if (!mark[c2[k]]) { mark[c2[k]] = 2; ++vote[2 * P + 1]; }
    }
    vote[2 * P + 1] += vote[2 * P];
    std::vector<uint8_t>().swap(mark);
    // the entries themselves, not only their counts: the split forms A[r,c] Q[c] on c's rank from
    // A[c,r], so p's tier-2 entries towards q must be q's tier-1 entries towards p transposed,
    // values included.  Per peer an order-free hash (wrapping sum of mixed (row, col, value
    // bits), tier 2 keyed transposed) is compared: a pattern or a value that is not symmetric
    // keeps the pull-all halo (or fails under RBL_OPT_HALO_PUSH 1) instead of a wrong SpMM.
    auto tier_hash = [&](int t, int64_t nz, const std::vector<int32_t>& cols, int64_t* out) -> int {
      if (nz == 0) return RBL_OK;
      std::vector<int64_t> trp(m + 1);
      std::vector<double> tv(nz);
      HIPC(hipMemcpy(trp.data(), ctx->seg_tier[t].rowptr, (m + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
      HIPC(hipMemcpy(tv.data(), ctx->seg_tier[t].val, nz * sizeof(double), hipMemcpyDeviceToHost));
      for (int64_t r = 0; r < m; ++r)
        for (int64_t k = trp[r]; k < trp[r + 1]; ++k) {
          const uint64_t row = (uint64_t)(ctx->r0 + r), col = (uint64_t)cols[k];
          uint64_t vb;
          memcpy(&vb, &tv[k], sizeof(vb));
          const uint64_t a = t == 1 ? row : col, b2 = t == 1 ? col : row;  // tier 2: transposed
          const uint64_t h = mix64(mix64(a * 0x9E3779B97F4A7C15ull ^ b2) ^ vb);
          out[owner(cols[k])] = (int64_t)((uint64_t)out[owner(cols[k])] + h);
        }
      return RBL_OK;
    };
    CHK(tier_hash(1, nz1, c1, vote.data() + 2 * P + 2));
    CHK(tier_hash(2, nz2, c2, vote.data() + 3 * P + 2));
    return RBL_OK;
  };
  const int lrc = local_counts();
  std::vector<int32_t>().swap(c2);
  const int V = 4 * P + 3;
  vote[4 * P + 2] = lrc;
  std::vector<int64_t> votes((size_t)P * V);
  COMMC(ctx->comm->allgather_host(vote.data(), votes.data(), V, ctx->stream, &ctx->err));
  if (lrc < 0) return lrc;  // (ctx->err already says what failed here)
  for (int p = 0; p < P; ++p)
    if (votes[(size_t)p * V + 4 * P + 2] < 0)
      return fail(ctx, (int)votes[(size_t)p * V + 4 * P + 2],
                  "push/pull halo setup failed on rank " + std::to_string(p));
  bool sym = true;
  int64_t d1 = 0, d12 = 0;
  for (int p = 0; p < P; ++p) {
    const int64_t* vp = votes.data() + (size_t)p * V;
    d1 += vp[2 * P];
    d12 += vp[2 * P + 1];
    for (int q = 0; q < P; ++q) {  // p's tier-2 entries towards q are q's tier-1 entries towards p
      const int64_t* vq = votes.data() + (size_t)q * V;
      if (vp[P + q] != vq[p] || vp[3 * P + 2 + q] != vq[2 * P + 2 + p]) sym = false;
    }
  }
  ctx->push_pred_rows = 2 * d1;
  ctx->pull_pred_rows = d12;
  if (!sym) {
    if (ctx->halo_push_opt == 1)
      return fail(ctx, RBL_ERR_INVALID, "RBL_OPT_HALO_PUSH: A is not symmetric (pattern or values)");
    return 0;
  }
  if (ctx->halo_push_opt == 2 && !(2.0 * (double)d1 < 0.85 * (double)d12)) return 0;
  // split: tier 2 dropped, the ghosts are tier 1's columns
  free_seg(ctx->seg_tier[2], true);
  ctx->seg_ntiers = 2;
  int32_t* d_map = nullptr;
  CHK(build_ghosts(ctx, &d_map, ctx->seg_tier[1].col, nz1));
  if (nz1) remap_cols(ctx->seg_tier[1].col, nz1, d_map, ctx->stream);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(ctx->stream));
  hipFree(d_map);
  ctx->seg_split = true;
  ctx->ghost = true;
  // the push tier: tier 1 transposed, rows = ghost slots (in row order within a slot)
  const int64_t G = ctx->n_ghost;
  std::vector<int64_t> rp1(m + 1, 0);
  std::vector<double> v1(std::max<int64_t>(nz1, 1));
  if (m > 0) HIPC(hipMemcpy(rp1.data(), ctx->seg_tier[1].rowptr, (m + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
  if (nz1) {
    HIPC(hipMemcpy(c1.data(), ctx->seg_tier[1].col, nz1 * sizeof(int32_t), hipMemcpyDeviceToHost));
    HIPC(hipMemcpy(v1.data(), ctx->seg_tier[1].val, nz1 * sizeof(double), hipMemcpyDeviceToHost));
  }
  std::vector<int64_t> prp(G + 1, 0);
  for (int64_t k = 0; k < nz1; ++k) ++prp[c1[k] + 1];
  for (int64_t g = 0; g < G; ++g) prp[g + 1] += prp[g];
  std::vector<int64_t> pos(prp.begin(), prp.end() - 1);
  std::vector<int32_t> pc(std::max<int64_t>(nz1, 1));
  std::vector<double> pv(std::max<int64_t>(nz1, 1));
  for (int64_t r = 0; r < m; ++r)
    for (int64_t k = rp1[r]; k < rp1[r + 1]; ++k) {
      const int64_t at = pos[c1[k]]++;
      pc[at] = (int32_t)(ctx->r0 + r);
      pv[at] = v1[k];
    }
  auto& T = ctx->push_tier;
  HIPC(hipMalloc(&T.rowptr, (G + 1) * sizeof(int64_t)));
  HIPC(hipMalloc(&T.col, (nz1 + kCsrPad) * sizeof(int32_t)));
  HIPC(hipMalloc(&T.val, (nz1 + kCsrPad) * sizeof(double)));
  HIPC(hipMemset(T.col, 0, (nz1 + kCsrPad) * sizeof(int32_t)));
  HIPC(hipMemset(T.val, 0, (nz1 + kCsrPad) * sizeof(double)));
  HIPC(hipMemcpy(T.rowptr, prp.data(), (G + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  if (nz1) {
    HIPC(hipMemcpy(T.col, pc.data(), nz1 * sizeof(int32_t), hipMemcpyHostToDevice));
    HIPC(hipMemcpy(T.val, pv.data(), nz1 * sizeof(double), hipMemcpyHostToDevice));
  }
  CHK(build_seg(ctx, prp, T));
  ctx->push_rows = G;
  // where the received partials go: the own rows asked for, each with its slots in peer order
  const int64_t ns = ctx->n_send;
  std::vector<int32_t> sidx(std::max<int64_t>(ns, 1));
  if (ns) HIPC(hipMemcpy(sidx.data(), ctx->d_send_idx, ns * sizeof(int32_t), hipMemcpyDeviceToHost));
  std::vector<int64_t> cnt(std::max<int64_t>(m, 1) + 1, 0);
  for (int64_t k = 0; k < ns; ++k) ++cnt[sidx[k] + 1];
  for (int64_t r = 0; r < m; ++r) cnt[r + 1] += cnt[r];
  std::vector<int64_t> slot(std::max<int64_t>(ns, 1)), rows, ptr(1, 0);
  {
    std::vector<int64_t> at(cnt.begin(), cnt.end() - 1);
    for (int64_t k = 0; k < ns; ++k) slot[at[sidx[k]]++] = k;
  }
  for (int64_t r = 0; r < m; ++r)
    if (cnt[r + 1] > cnt[r]) {
      rows.push_back(r);
      ptr.push_back(cnt[r + 1]);
    }
  ctx->n_ps_rows = (int64_t)rows.size();
  HIPC(hipMalloc(&ctx->d_ps_rows, std::max<size_t>(rows.size(), 1) * sizeof(int64_t)));
  HIPC(hipMalloc(&ctx->d_ps_ptr, ptr.size() * sizeof(int64_t)));
  HIPC(hipMalloc(&ctx->d_ps_slot, slot.size() * sizeof(int64_t)));
  if (!rows.empty())
    HIPC(hipMemcpy(ctx->d_ps_rows, rows.data(), rows.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  HIPC(hipMemcpy(ctx->d_ps_ptr, ptr.data(), ptr.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  HIPC(hipMemcpy(ctx->d_ps_slot, slot.data(), slot.size() * sizeof(int64_t), hipMemcpyHostToDevice));
  ctx->push = true;
  return 1;
}

// Column tiers of the segmented gather (RBL_SEG_TIERS="h[,w]": the h highest-degree columns,
// then the next w, then the rest; one rank, A symmetric so a column's degree is its row's).
// The SpMM sweeps the tiers in order; each sweep's gathers hit a Q-row set sized for one cache
// level.  Results differ from the one-sweep SpMM only in the order of each row's sum.
// Several ranks (unbanded A, the segmented gather): two tiers instead, the own columns
// [r0, r1) and the halo columns, so the own part of the SpMM runs while the halo exchange is in
// flight (step_impl); the sum order per row is the same with or without the overlap.
// the column panels on several ranks need the range halo: taken where every block's window
// is a small part of the matrix (a band), not where the windows span it (a small R-MAT's blocks
// may pass panel_auto, and its indexed halo moves fewer rows)
bool panel_banded(const rbl_ctx* ctx) { return ctx->panel_auto && 4 * ctx->panel_span <= ctx->n; }

int prepare_tiers(rbl_ctx* ctx, const std::vector<int64_t>& rp) {
  free_tiers(ctx);
  ctx->push_pred_rows = ctx->pull_pred_rows = 0;
  if (ctx->nranks > 1) {
    // every rank must take the same branch (the setup below runs collectives), so the vote
    // comes before any per-rank condition: a rank with no rows or no nonzeros still takes
    // part in build_ghosts (with no requests), and a rank that released its CSR for band tiles
    // (RBL_OPT_KEEP_CSR = 0) votes banded, which stops every rank here
    const int64_t banded = (ctx->bt_ng || ctx->band_ok16 || ctx->band_ok32 || ctx->window_ok16 ||
                            ctx->window_ok32 || panel_banded(ctx) || ctx->dense || ctx->csr_dropped)
                               ? 1 : 0;
    std::vector<int64_t> all(ctx->nranks);
    COMMC(ctx->comm->allgather_host(&banded, all.data(), 1, ctx->stream, &ctx->err));
    for (int64_t v : all)
      if (v) return RBL_OK;  // a banded kernel runs: its halo is a range of rows
    std::vector<uint8_t> tier_of(ctx->n, 1);
    for (int64_t c = ctx->r0; c < ctx->r1; ++c) tier_of[c] = 0;
    if (ctx->halo_push_opt != 0) {  // the push/pull split, if it moves fewer rows (collective)
      const int ps = prepare_push(ctx, rp);
      if (ps < 0) return ps;
      if (ps == 1) return RBL_OK;
      free_tiers(ctx);
    }
    int32_t* d_map = nullptr;
    CHK(build_ghosts(ctx, &d_map, ctx->d_col, ctx->nnz));
    const int st = build_tiers(ctx, tier_of, 2);
    if (st == RBL_OK) {
      remap_cols(ctx->seg_tier[1].col, ctx->seg_tier[1].ntasks > 0 ? tier_nnz(ctx, 1) : 0, d_map,
                 ctx->stream);
      HIPC(hipGetLastError());
      HIPC(hipStreamSynchronize(ctx->stream));
    }
    hipFree(d_map);
    CHK(st);
    ctx->seg_split = true;
    ctx->ghost = true;
    // the rows this halo moves per SpMM, summed over ranks (rbl_comm_stats' halo plan)
    std::vector<int64_t> ng(ctx->nranks);
    COMMC(ctx->comm->allgather_host(&ctx->n_ghost, ng.data(), 1, ctx->stream, &ctx->err));
    ctx->pull_pred_rows = 0;
    for (int64_t v : ng) ctx->pull_pred_rows += v;
    return RBL_OK;
  }
  if (ctx->seg_ntasks == 0 || ctx->nnz == 0 || ctx->csr_dropped) return RBL_OK;
#ifndef RBL_VARIANTS
  return RBL_OK;
#else
  // (variants build only: the degree-ranked column tiers of one rank, measured no faster,
  // DESIGN.md §3 round 3)
  const char* e = std::getenv("RBL_SEG_TIERS");
  if (!e || ctx->nloc != ctx->n) return RBL_OK;
  std::vector<int64_t> sz;
  for (const char* p = e; *p;) {
    char* end = nullptr;
    const long long v = std::strtoll(p, &end, 10);
    if (end == p) break;
    if (v > 0) sz.push_back(v);
    p = *end == ',' ? end + 1 : end;
    if (sz.size() == kMaxSegTiers - 1) break;
  }
  if (sz.empty()) return RBL_OK;
  const int nt = (int)sz.size() + 1;
  const int64_t n = ctx->n, m = ctx->nloc;
  std::vector<int64_t> order(n);
  for (int64_t c = 0; c < n; ++c) order[c] = c;
  std::stable_sort(order.begin(), order.end(), [&](int64_t a, int64_t b2) {
    return rp[a + 1] - rp[a] > rp[b2 + 1] - rp[b2];
  });
  std::vector<uint8_t> tier_of(n, (uint8_t)(nt - 1));
  int64_t rank = 0;
  for (int t = 0; t < nt - 1; ++t)
    for (int64_t k = 0; k < sz[t] && rank < n; ++k) tier_of[order[rank++]] = (uint8_t)t;
  (void)m;
  return build_tiers(ctx, tier_of, nt);
#endif
}

// The tier CSRs and task tables for a column -> tier map (tier_of: n entries, < nt), or for
// the per-nonzero rule of the push/pull halo split (rule, nt = 3).
int build_tiers(rbl_ctx* ctx, const std::vector<uint8_t>& tier_of, int nt, const TierRule* rule) {
  const int64_t n = ctx->n, m = ctx->nloc;
  uint8_t* d_tier = nullptr;
  int32_t* d_cnt = nullptr;
  HIPC(hipMalloc(&d_tier, rule ? 1 : n));
  HIPC(hipMalloc(&d_cnt, std::max<size_t>((size_t)nt * m, 1) * sizeof(int32_t)));
  if (rule)
    seg_tier_count_rule(m, ctx->d_rowptr, ctx->d_col, *rule, d_cnt, ctx->stream);
  else {
    HIPC(hipMemcpy(d_tier, tier_of.data(), n, hipMemcpyHostToDevice));
    seg_tier_count(m, ctx->d_rowptr, ctx->d_col, d_tier, nt, d_cnt, ctx->stream);
  }
  HIPC(hipGetLastError());
  std::vector<int32_t> cnt((size_t)nt * m);
  HIPC(hipMemcpyAsync(cnt.data(), d_cnt, cnt.size() * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  std::vector<std::vector<int64_t>> trp(nt, std::vector<int64_t>(m + 1, 0));
  int64_t* rpp[kMaxSegTiers] = {nullptr, nullptr, nullptr};
  int32_t* colp[kMaxSegTiers] = {nullptr, nullptr, nullptr};
  double* valp[kMaxSegTiers] = {nullptr, nullptr, nullptr};
  for (int t = 0; t < nt; ++t) {
    for (int64_t r = 0; r < m; ++r) trp[t][r + 1] = trp[t][r] + cnt[(size_t)t * m + r];
    auto& T = ctx->seg_tier[t];
    const int64_t nz = trp[t][m];
    HIPC(hipMalloc(&T.rowptr, (m + 1) * sizeof(int64_t)));
    HIPC(hipMalloc(&T.col, (nz + kCsrPad) * sizeof(int32_t)));
    HIPC(hipMalloc(&T.val, (nz + kCsrPad) * sizeof(double)));
    HIPC(hipMemset(T.col + nz, 0, kCsrPad * sizeof(int32_t)));
    HIPC(hipMemset(T.val + nz, 0, kCsrPad * sizeof(double)));
    HIPC(hipMemcpy(T.rowptr, trp[t].data(), (m + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
    rpp[t] = T.rowptr;
    colp[t] = T.col;
    valp[t] = T.val;
  }
  ctx->seg_ntiers = nt;  // (free_tiers releases partial state on a later failure)
  if (rule)
    seg_tier_fill_rule(m, ctx->d_rowptr, ctx->d_col, ctx->d_val, *rule, rpp, colp, valp, ctx->stream);
  else
    seg_tier_fill(m, ctx->d_rowptr, ctx->d_col, ctx->d_val, d_tier, nt, rpp, colp, valp, ctx->stream);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(ctx->stream));
  hipFree(d_tier);
  hipFree(d_cnt);
  for (int t = 0; t < nt; ++t) {
    auto& T = ctx->seg_tier[t];
    int64_t* rp_keep = T.rowptr;
    int32_t* col_keep = T.col;
    double* val_keep = T.val;
    CHK(build_seg(ctx, trp[t], T));
    T.rowptr = rp_keep;
    T.col = col_keep;
    T.val = val_keep;
  }
  return RBL_OK;
}

// Per-16-row-tile column footprint for the LDS-window SpMM and the checks that every tile
// fits its ring (spmm_window.hip): columns sorted per row, footprints non-decreasing, a
// tile's nonzeros <= 2048, ring rows: 256 (b=32) / 512 (b=16), new rows per tile <= 32 / 64.
int prepare_window_formats(rbl_ctx* ctx, const std::vector<int64_t>& rp);
// the column-panel SpMM's limit: panels per row block (256-row panels: windows <= 16 K rows)
constexpr int64_t kPanelMax = 64;
// Every SpMM format of a freshly set CSR: the segmented-gather table, the window / band /
// band-tile formats, then (unbanded only) the column tiers.
int prepare_window(rbl_ctx* ctx, const std::vector<int64_t>& rp) {
  CHK(prepare_window_formats(ctx, rp));
  CHK(prepare_tiers(ctx, rp));  // (collective on several ranks: every rank calls it)
  return RBL_OK;
}

int prepare_window_formats(rbl_ctx* ctx, const std::vector<int64_t>& rp) {
  CHK(prepare_segments(ctx, rp));
  ctx->window_ok16 = ctx->window_ok32 = false;
  ctx->band_ok16 = ctx->band_ok32 = false;
  ctx->band_gram = false;
  ctx->band_pair = false;
  ctx->ntiles = (ctx->nloc + kWindowTileRows - 1) / kWindowTileRows;
  if (ctx->ntiles == 0 || ctx->nnz == 0) return RBL_OK;
  const int64_t nt = ctx->ntiles;
  HIPC(hipMalloc(&ctx->d_tcmin, nt * sizeof(int64_t)));
  HIPC(hipMalloc(&ctx->d_tcmax, nt * sizeof(int64_t)));
  CsrDev A;
  A.nrows = ctx->nloc;
  A.rowptr = ctx->d_rowptr;
  A.col = ctx->d_col;
  tile_col_range(A, kWindowTileRows, ctx->d_tcmin, ctx->d_tcmax, ctx->stream);
  std::vector<int64_t> cmin(nt), cmax(nt);
  HIPC(hipMemcpyAsync(cmin.data(), ctx->d_tcmin, nt * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipMemcpyAsync(cmax.data(), ctx->d_tcmax, nt * sizeof(int64_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  // band-tile kernel (spmm_bt.hip): every nonempty tile's columns within
  // [r0 + 16t - H, r0 + 16t + 16 + H) for H = 32 or 64
  int64_t hneed = 0;
  for (int64_t t = 0; t < nt; ++t) {
    if (cmax[t] < 0) continue;
    const int64_t ra = ctx->r0 + t * kWindowTileRows;
    hneed = std::max(hneed, std::max(ra - cmin[t], cmax[t] - (ra + kWindowTileRows - 1)));
  }
  // forward-fill empty tiles (cmax < 0), then backward-fill leading empties
  int64_t first = -1;
  for (int64_t t = 0; t < nt; ++t) {
    if (cmax[t] < 0) {
      if (t > 0) { cmin[t] = cmin[t - 1]; cmax[t] = cmax[t - 1]; }
    } else if (first < 0) {
      first = t;
    }
  }
  if (first < 0) return RBL_OK;
  for (int64_t t = 0; t < first; ++t) { cmin[t] = cmin[first]; cmax[t] = cmax[first]; }
  bool ok = true;
  int64_t max_span = 0, max_new = 0;
  for (int64_t t = 0; t < nt && ok; ++t) {
    const int64_t ra = t * kWindowTileRows;
    const int64_t rb = std::min(ra + kWindowTileRows, ctx->nloc);
    if (rp[rb] - rp[ra] > 2048) ok = false;
    max_span = std::max(max_span, cmax[t] + 1 - cmin[t]);
    if (t > 0) {
      if (cmin[t] < cmin[t - 1] || cmax[t] < cmax[t - 1]) ok = false;
      max_span = std::max(max_span, cmax[t] + 1 - cmin[t - 1]);
      max_new = std::max(max_new, cmax[t] - std::max(cmax[t - 1], cmin[t] - 1));
    }
  }
  ctx->window_ok32 = ok && max_span <= 256 && max_new <= 32;
  ctx->window_ok16 = ok && max_span <= 512 && max_new <= 64;
  // band (MFMA) kernel (spmm_band.hip): tile band [c16, cmax] (c16 = cmin & ~15) at most
  // kBandMaxK columns, rows <= 192 nonzeros, and the dense tiles at least 25 % filled (else
  // the zero padding costs more than it saves)
  {
    int64_t max_row = 0, dense = 0, max_k = 0;
    for (int64_t i = 0; i < ctx->nloc; ++i) max_row = std::max(max_row, rp[i + 1] - rp[i]);
    for (int64_t t = 0; t < nt; ++t) {
      const int64_t k = cmax[t] + 1 - (cmin[t] & ~int64_t(15));
      max_k = std::max(max_k, k);
      dense += kWindowTileRows * ((k + 15) / 16 * 16);
    }
    // producers write tile t+2's new ring rows while tile t is multiplied: the ring must hold
    // [cmin(t), cmax(t+2)]
    int64_t max_span2 = 0;
    for (int64_t t = 0; t < nt; ++t)
      max_span2 = std::max(max_span2, cmax[std::min(t + 2, nt - 1)] + 1 - cmin[t]);
    const bool bok = ok && max_span2 <= kBandRing && max_k <= kBandMaxK && max_row <= 192 &&
                     4 * ctx->nnz >= dense;
    ctx->band_ok32 = bok && max_new <= 32;
    ctx->band_ok16 = bok && max_new <= 64;
    // A_i = Q^T U inside the band kernel reads Q's tile rows from the ring: each tile's own
    // (global) rows must lie in its band, and stay resident until the tile's U is final (one
    // phase late at b=16): rows [r(t), r(t)+16) vs the ring's [cmin(t), cmax(t+3)]
    bool gok = bok;
    for (int64_t t = 0; t < nt && gok; ++t) {
      const int64_t ra = ctx->r0 + t * kWindowTileRows;
      const int64_t rb = ctx->r0 + std::min((t + 1) * kWindowTileRows, ctx->nloc) - 1;
      if (ra < cmin[t] || rb > cmax[t]) gok = false;
      if (cmax[std::min(t + 3, nt - 1)] + 1 - ra > kBandRing) gok = false;
    }
    ctx->band_gram = gok;
    // rows (2p, 2p+1) of every 16-row tile: nonzeros + up to 3 of alignment shift <= 256
    int64_t max_pair = 0;
    for (int64_t r = 0; r < ctx->nloc; r += 2)
      max_pair = std::max(max_pair, rp[std::min(r + 2, ctx->nloc)] - rp[r]);
    ctx->band_pair = bok && max_pair + 3 <= 256;
  }
  HIPC(hipMemcpy(ctx->d_tcmin, cmin.data(), nt * sizeof(int64_t), hipMemcpyHostToDevice));
  HIPC(hipMemcpy(ctx->d_tcmax, cmax.data(), nt * sizeof(int64_t), hipMemcpyHostToDevice));
  std::vector<int64_t> info(8 * nt, 0);
  for (int64_t t = 0; t < nt; ++t) {
    const int64_t ra = t * kWindowTileRows;
    const int64_t rb = std::min(ra + kWindowTileRows, ctx->nloc);
    int64_t lo = cmin[t];
    if (t > 0) lo = std::max(lo, cmax[t - 1] + 1);
    const int64_t hi = std::max(lo, cmax[t] + 1);
    int64_t* f = &info[8 * t];
    f[0] = rp[ra];
    f[1] = rp[rb] - rp[ra];
    f[2] = lo;
    f[3] = hi;
    f[4] = cmin[t];
    f[5] = cmax[t];
  }
  HIPC(hipMalloc(&ctx->d_tinfo, 8 * nt * sizeof(int64_t)));
  HIPC(hipMemcpy(ctx->d_tinfo, info.data(), 8 * nt * sizeof(int64_t), hipMemcpyHostToDevice));
  const int64_t grid = window_grid();
  ctx->tiles_per_wg = std::max<int64_t>(1, (nt + grid - 1) / grid);
  {
    // dense tiles of 16 x (16 + 2H) doubles pay when they stream no more than ~1.25x the
    // CSR's values + column indices (C4a: 18.4 KB vs 19.2 KB per tile)
    const int H = hneed <= 32 ? 32 : hneed <= 64 ? 64 : 0;
    const int NG = H ? (2 * H + 16) / 16 : 0;
    const double dense_bytes = (double)nt * 16.0 * 16.0 * NG * 8.0;
    if (H && dense_bytes <= 1.25 * 12.0 * (double)ctx->nnz) {
      const size_t elems = (size_t)bt_tile_slots(nt, ctx->tiles_per_wg) * NG * 256;
      HIPC(hipMalloc(&ctx->d_bt, elems * sizeof(double)));
      HIPC(hipMemsetAsync(ctx->d_bt, 0, elems * sizeof(double), ctx->stream));
      if (!ctx->d_zrow) {
        HIPC(hipMalloc(&ctx->d_zrow, 64 * sizeof(double)));
        HIPC(hipMemsetAsync(ctx->d_zrow, 0, 64 * sizeof(double), ctx->stream));
      }
      CsrDev A3 = csr(ctx);
      bt_fill(A3, H, NG, ctx->d_bt, ctx->stream);
      HIPC(hipGetLastError());
      HIPC(hipStreamSynchronize(ctx->stream));
      ctx->bt_ng = NG;
#ifdef RBL_VARIANTS
      // (variants build only) RBL_BT_PACK = 1: pack the tiles (zeros dropped; C4a: 13.1 KB per tile instead of
      // 18.4 KB, 3 GB less HBM at n = 1e7).  Off by default: the kernel is not bound by its
      // A bytes (one wave per SIMD, 60 % MFMA busy, fp64 MFMA and VALU do not co-issue) and
      // the index arithmetic of the packed loads costs more than the bytes save (3.56 vs
      // 3.40 ms per launch at C4a)
      const char* pk = getenv("RBL_BT_PACK");
      if (pk && atoi(pk) == 1) {
        const int64_t nslots = bt_tile_slots(nt, ctx->tiles_per_wg);
        HIPC(hipMalloc(&ctx->d_btp_hdr, (size_t)nslots * bt_pack_words(NG) * sizeof(uint64_t)));
        int64_t nval = 0;
        const int prc = bt_pack(ctx->d_bt, nslots, NG, ctx->d_btp_hdr, &ctx->d_btp_val, &nval, ctx->stream);
        if (prc != 0) return prc == (int)hipErrorOutOfMemory ? RBL_ERR_OOM : RBL_ERR_HIP;
        hipFree(ctx->d_bt);
        ctx->d_bt = nullptr;
      } else {
        // A symmetric (bit for bit, as Lanczos assumes): store the diagonal group and the
        // right strip only — 10 of 18.4 KB per tile at H = 64; the kernel transposes the left
        // groups back from the previous tiles' strips (same U bits).  Opt-in (RBL_BT_HALF = 1)
        // while it measures slower than the whole tiles.
        const char* hf = getenv("RBL_BT_HALF");
        if (hf && atoi(hf) == 1) {
          double *half = nullptr, *edge = nullptr;
          const int hrc = bt_half(ctx->d_bt, nt, ctx->tiles_per_wg, NG, &half, &edge, ctx->stream);
          if (hrc > 0) return hrc == (int)hipErrorOutOfMemory ? RBL_ERR_OOM : RBL_ERR_HIP;
          if (hrc == 0) {
            hipFree(ctx->d_bt);
            ctx->d_bt = nullptr;
            ctx->d_bth = half;
            ctx->d_bte = edge;
          }
        }
      }
#endif
    }
  }
  // column-panel SpMM (spmm_panel.hip; not when the band tiles serve the matrix): per block of
  // R = 64 rpg rows the panels its columns span and every row's count in each of them;
  // applicable when no block spans more than kPanelMax panels (a window of 16 K rows: beyond
  // that the panels' re-reads cost more than the gathers they replace)
  if (!ctx->bt_ng) {
    const int pw = panel_width();
    // 8 rows per group (16-entry chunks) when a row's count per panel is mostly small, else 4
    // (32-entry chunks): the mean count per row and panel at 512-row blocks decides
    auto plan = [&](int R, std::vector<int32_t>* bp, int64_t* maxp, int64_t* staged) {
      const int tpb = R / kWindowTileRows;
      const int64_t nb = (nt + tpb - 1) / tpb;
      if (bp) bp->assign(4 * nb, 0);
      *maxp = *staged = 0;
      int64_t coff = 0;
      for (int64_t bk = 0; bk < nb; ++bk) {
        int64_t lo = INT64_MAX, hi = -1;
        for (int64_t t = bk * tpb; t < std::min(nt, (bk + 1) * tpb); ++t) {
          lo = std::min(lo, cmin[t]);
          hi = std::max(hi, cmax[t]);
        }
        const int64_t np = hi / pw - lo / pw + 1;
        if (bp) {
          (*bp)[4 * bk] = (int32_t)(lo / pw);
          (*bp)[4 * bk + 1] = (int32_t)(hi / pw);
          (*bp)[4 * bk + 2] = (int32_t)(uint32_t)(coff & 0xffffffff);
          (*bp)[4 * bk + 3] = (int32_t)(coff >> 32);
        }
        coff += np * R;
        *maxp = std::max(*maxp, np);
        *staged += np * pw;
      }
      return nb;
    };
    int64_t maxp = 0, staged = 0;
    plan(512, nullptr, &maxp, &staged);
    // the kernel's shape by the mean count per row and panel at 512-row blocks: 8 rows per
    // group with 16-record chunks up to a mean of 16, else 4 rows per group with 48-record
    // chunks (the three shapes forced at H = 128..2048: profiles/r06_panel_shapes_b30.txt)
    const double mean_cnt = (double)ctx->nnz / std::max(1.0, (double)(staged / pw) * 512);
#ifdef RBL_PANEL_RPG  // (probe builds: tools/build_variant.sh-style A/B of the kernel shape)
    const int rpg = RBL_PANEL_RPG, pch = RBL_PANEL_CH;
#else
    const int rpg = mean_cnt <= 16.0 ? 8 : 4;
    const int pch = rpg == 8 ? 16 : 48;
#endif
    const int R = 64 * rpg;
    std::vector<int32_t> bp;
    const int64_t nb = plan(R, &bp, &maxp, &staged);
    const int64_t ncnt = bp.empty() ? 0 : ((int64_t)(uint32_t)bp[4 * nb - 2] | ((int64_t)bp[4 * nb - 1] << 32)) +
                                              ((int64_t)bp[4 * nb - 3] - bp[4 * nb - 4] + 1) * R;
    // the kernel addresses a block's records with 32-bit buffer offsets: every block's
    // values within 2 GiB (the block bases, rowptr[b R], read strided)
    int64_t maxblk = 0;
    if (maxp <= kPanelMax && ctx->n / pw < INT32_MAX && nb > 0) {
      std::vector<int64_t> zb(nb + 1);
      HIPC(hipMemcpy2D(zb.data(), sizeof(int64_t), ctx->d_rowptr, (size_t)R * sizeof(int64_t),
                       sizeof(int64_t), (size_t)nb, hipMemcpyDeviceToHost));
      zb[nb] = ctx->nnz;
      for (int64_t bk = 0; bk < nb; ++bk) maxblk = std::max(maxblk, zb[bk + 1] - zb[bk]);
    }
    bool fits = maxp <= kPanelMax && ctx->n / pw < INT32_MAX && nb > 0 && maxblk * 8 < INT32_MAX;
    // the records are a second copy of the matrix: without room for it, no panels (the gathers).
    // An allocation that fails here is not an error: this rank just runs another kernel (the
    // several-rank setup after this is collective, so no rank may leave before it)
    if (fits) {
      const bool ok =
          hipMalloc(&ctx->d_panel_val, std::max<int64_t>(ctx->nnz, 1) * sizeof(double)) == hipSuccess &&
          hipMalloc(&ctx->d_panel_col, std::max<int64_t>(ctx->nnz, 1)) == hipSuccess &&
          hipMalloc(&ctx->d_panel_blk, 4 * nb * sizeof(int32_t)) == hipSuccess &&
          hipMalloc(&ctx->d_panel_cnt, std::max<int64_t>(ncnt, 1) * sizeof(uint16_t)) == hipSuccess &&
          hipMalloc(&ctx->d_panel_st, std::max<int64_t>(ncnt, 1) * sizeof(uint32_t)) == hipSuccess;
      if (!ok) {
        (void)hipGetLastError();
        free_panels(ctx);
        fits = false;
      }
    }
    if (fits) {
      HIPC(hipMemcpy(ctx->d_panel_blk, bp.data(), 4 * nb * sizeof(int32_t), hipMemcpyHostToDevice));
      CsrDev A2 = csr(ctx);
      if (panel_format(A2, ctx->d_panel_blk, R, nb, ctx->d_panel_cnt, ctx->d_panel_st, ncnt,
                       ctx->d_panel_col, ctx->d_panel_val, ctx->stream) != 0)
        return fail(ctx, RBL_ERR_HIP, "panel_format");
      HIPC(hipStreamSynchronize(ctx->stream));
      ctx->panel_nblk = nb;
      ctx->panel_rpg = rpg;
      ctx->panel_ch = pch;
      // by default only where the panels pay: a staged Q row read >= 4 times from LDS on
      // average (bands; a scattered pattern's blocks span the whole matrix: the gathers).  Ahead
      // of the LDS-window kernel where both apply: 5.0 vs 7.6 ms at H = 72 and 96, n = 1e7
      // (profiles/r06_panel_vs_window_b19.txt)
      ctx->panel_auto = 4 * staged <= ctx->nnz;
      ctx->panel_span = maxp * pw;
      if (!ctx->d_zrow) {  // the panel rows outside the Q range read it
        HIPC(hipMalloc(&ctx->d_zrow, 64 * sizeof(double)));
        HIPC(hipMemset(ctx->d_zrow, 0, 64 * sizeof(double)));
      }
    }
  }
  if (!ctx->keep_csr && ctx->bt_ng) {
    // RBL_OPT_KEEP_CSR = 0: the band tiles are the matrix from here on
    hipFree(ctx->d_col); ctx->d_col = nullptr;
    hipFree(ctx->d_val); ctx->d_val = nullptr;
    hipFree(ctx->d_seg_trow); ctx->d_seg_trow = nullptr;
    hipFree(ctx->d_seg_tinfo); ctx->d_seg_tinfo = nullptr;
    hipFree(ctx->d_seg_slot_k0); ctx->d_seg_slot_k0 = nullptr;
    hipFree(ctx->d_seg_lrow); ctx->d_seg_lrow = nullptr;
    hipFree(ctx->d_seg_lslot); ctx->d_seg_lslot = nullptr;
    hipFree(ctx->d_seg_scratch); ctx->d_seg_scratch = nullptr;
    ctx->seg_ntasks = ctx->seg_nlong = 0;
    free_tiers(ctx);
    ctx->window_ok16 = ctx->window_ok32 = false;
    ctx->band_ok16 = ctx->band_ok32 = false;
    ctx->band_gram = ctx->band_pair = false;
    ctx->csr_dropped = true;
    return RBL_OK;
  }
  if (ctx->band_ok16 || ctx->band_ok32) {  // dense-tile positions for the band kernel
    HIPC(hipMalloc(&ctx->d_bpos, (ctx->nnz + kCsrPad) * sizeof(uint16_t)));
    HIPC(hipMemsetAsync(ctx->d_bpos + ctx->nnz, 0, kCsrPad * sizeof(uint16_t), ctx->stream));
    CsrDev A2 = csr(ctx);
    band_positions(A2, ctx->d_bpos, ctx->stream);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(ctx->stream));
  }
  return RBL_OK;
}

// ---- timers --------------------------------------------------------------------------
hipEvent_t next_event(rbl_ctx* ctx) {
  if (ctx->ev_used == ctx->ev_pool.size()) {
    hipEvent_t e;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    ctx->ev_pool.push_back(e);
  }
  return ctx->ev_pool[ctx->ev_used++];
}
struct StageScope {
  rbl_ctx* ctx;
  int stage;
  hipEvent_t a = nullptr;
  // every stage is also a roctx range named like the reference's TimerOutputs labels
  // (RBL_gpu.jl:152-187: "AQ", "3-term", ...): `rocprofv3 --marker-trace` shows them
  hipStream_t st;
  int parent = -1;
  StageScope(rbl_ctx* c, int s, hipStream_t on = nullptr) : ctx(c), stage(s), st(on ? on : c->stream) {
    roctxRangePushA(kStageNames[s]);
    if (ctx->timers == 1 ||
        (ctx->timers == 2 && (s == RBL_STAGE_AQ || s == RBL_STAGE_PART_REORTH))) {
      a = next_event(ctx);
      if (a) hipEventRecord(a, st);
    }
    // a collective issued inside another stage on the same stream: its span is "comm" only, so
    // the stages of a step sum to the step's stream time (the multi-rank line's per-rank split)
    if (s == RBL_STAGE_COMM)
      for (auto it = ctx->open_stages.rbegin(); it != ctx->open_stages.rend(); ++it)
        if (it->st == st) {
          parent = it->stage;
          break;
        }
    ctx->open_stages.push_back({s, st});
  }
  ~StageScope() {
    ctx->open_stages.pop_back();
    if (a) {
      hipEvent_t b = next_event(ctx);
      if (b) {
        hipEventRecord(b, st);
        ctx->marks.push_back({stage, a, b, parent});
      }
    }
    roctxRangePop();
  }
};
void harvest_timers(rbl_ctx* ctx) {
  // stages whose end event has completed; the rest (steps still running after an rbl_fetch
  // that waited only for earlier steps) stay for a later harvest, their events in use
  std::vector<rbl_ctx::Mark> keep;
  for (auto& m : ctx->marks) {
    if (hipEventQuery(m.b) != hipSuccess) {
      keep.push_back(m);
      continue;
    }
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, m.a, m.b) == hipSuccess) {
      if (m.stage < RBL_NUM_STAGES) {
        ctx->stage_ms[m.stage] += ms;
        if (m.parent >= 0) ctx->stage_ms[m.parent] -= ms;  // (recorded whenever the child is)
      } else {
        ctx->comm_dev_ms[m.stage - RBL_NUM_STAGES] += ms;  // a CollScope's span
      }
    }
  }
  ctx->marks.swap(keep);
  if (ctx->marks.empty()) ctx->ev_used = 0;
}

// ---- collectives ---------------------------------------------------------------------
// One collective call: the host wall time inside the transport (RCCL enqueues and returns;
// the shm / in-process stand-ins block) and, while the full stage timers run, a hipEvent pair
// around it on its stream — the span the collective holds that stream, waiting for the peers
// included.  Read per rank through rbl_comm_stats (RBL_COMM_*_HOST_NS / *_DEV_NS).
struct CollScope {
  rbl_ctx* ctx;
  int kind;  // 0 all-reduce, 1 exchange
  hipStream_t st;
  hipEvent_t a = nullptr;
  std::chrono::steady_clock::time_point t0;
  CollScope(rbl_ctx* c, int k, hipStream_t on) : ctx(c), kind(k), st(on) {
    if (ctx->timers == 1) {
      a = next_event(ctx);
      if (a) hipEventRecord(a, st);
    }
    t0 = std::chrono::steady_clock::now();
  }
  ~CollScope() {
    ctx->comm_host_ns[kind] += std::chrono::duration_cast<std::chrono::nanoseconds>(
                                   std::chrono::steady_clock::now() - t0).count();
    if (a) {
      hipEvent_t b = next_event(ctx);
      if (b) {
        hipEventRecord(b, st);
        ctx->marks.push_back({RBL_NUM_STAGES + kind, a, b});
      }
    }
  }
};

int allreduce(rbl_ctx* ctx, double* buf, size_t count) {
  if (ctx->nranks == 1) return RBL_OK;
  StageScope t(ctx, RBL_STAGE_COMM);
  CollScope c(ctx, 0, ctx->stream);
  COMMC(ctx->comm->allreduce_sum(buf, count, ctx->stream, &ctx->err));
  ctx->comm_stats[RBL_COMM_ALLREDUCE_CALLS] += 1;
  ctx->comm_stats[RBL_COMM_ALLREDUCE_BYTES] += (int64_t)(count * sizeof(double));
  return RBL_OK;
}

void count_exchange(rbl_ctx* ctx, const std::vector<Comm::Xfer>& x) {
  ctx->comm_stats[RBL_COMM_EXCHANGE_CALLS] += 1;
  for (const auto& t : x) {
    ctx->comm_stats[RBL_COMM_SEND_BYTES] += (int64_t)(t.nsend * sizeof(double));
    ctx->comm_stats[RBL_COMM_RECV_BYTES] += (int64_t)(t.nrecv * sizeof(double));
  }
}

// a step's grouped halo send/recv on `st`, timed and counted
int exchange(rbl_ctx* ctx, const std::vector<Comm::Xfer>& x, hipStream_t st) {
  CollScope c(ctx, 1, st);
  COMMC(ctx->comm->exchange(x, st, &ctx->err));
  count_exchange(ctx, x);
  return RBL_OK;
}

// Gram C = W^T X over all ranks.  C layout [nW*w][X.count*X.w].  (comm = false: this rank's
// share only, for a caller that all-reduces it together with another buffer)
int gram(rbl_ctx* ctx, const PanelRun& W, const Panels& X, double* C, const int* skip, bool comm = true) {
  const int xcols = X.count * X.w;
  const int splits = gram_splits(ctx->nloc, W.count, W.w, xcols);
  const int64_t len = (int64_t)W.count * W.w * xcols;
  if ((size_t)splits * len > ctx->slab_elems)
    return fail(ctx, RBL_ERR_INVALID, "internal: Gram slab too small");
  if (ctx->nloc > 0) {
    gram_partial(ctx->nloc, W, X, ctx->d_slab, splits, skip, ctx->stream);
    reduce_slab(ctx->d_slab, splits, len, C, skip, ctx->stream);
  } else {
    HIPC(hipMemsetAsync(C, 0, len * sizeof(double), ctx->stream));
  }
  HIPC(hipGetLastError());
  return comm ? allreduce(ctx, C, (size_t)len) : RBL_OK;
}

PanelRun run1(const double* p, int w) {
  PanelRun r;
  r.base = p;
  r.stride = 0;
  r.count = 1;
  r.w = w;
  return r;
}
Panels pan1(const double* p, int w) {
  Panels x;
  x.ptr[0] = p;
  x.count = 1;
  x.w = w;
  return x;
}
Panels pan2(const double* p0, const double* p1, int w) {
  Panels x;
  x.ptr[0] = p0;
  x.ptr[1] = p1;
  x.count = 2;
  x.w = w;
  return x;
}

// small-buffer carve (b x b each)
// S_CHS*: chol scratch (b > 64); S_RINV1: R1^-1 kept for the 3-pass CholQR; S_CLOC: the next
// step's local-reorth Gram
// (S_CLOC follows S_G: CholQR's pass-3 Gram and the next step's local-reorth Gram share one
// all-reduce of 2 b^2)
enum { S_R = 0, S_RINV, S_RTOT, S_BPREV, S_AI, S_G, S_CLOC, S_BT, S_CHS0, S_CHS1, S_RINV1, S_NSMALL };
static_assert(S_CLOC == S_G + 1, "tsqr all-reduces [S_G | S_CLOC] as one 2 b^2 buffer");
double* smallp(rbl_ctx* ctx, int which) { return ctx->d_small + (int64_t)which * ctx->b * ctx->b; }

int tsmm_checked(rbl_ctx* ctx, const PanelRun& X, const double* C, int ldc, const Panels& Y,
                 double alpha, double beta, const int* skip, double* xslab = nullptr,
                 int* xgrid = nullptr) {
  if (xgrid) *xgrid = 0;
  if (ctx->nloc <= 0) return RBL_OK;
  tsmm(ctx->nloc, X, C, ldc, Y, alpha, beta, skip, ctx->stream, xslab, xgrid);
  HIPC(hipGetLastError());
  return RBL_OK;
}

// Fused one-pass row operation (rowop.hip): Y = beta Y + alpha X C and, if G, the Gram
// G = Y^T Y over all ranks.  b in {16, 32}.
int rowop(rbl_ctx* ctx, const double* X, const double* C, double* Y, double alpha, double beta,
          double* G, const int* skip, const float* X32 = nullptr, float* Y32 = nullptr,
          const int* f64flag = nullptr, bool tri = false) {
  const int b = ctx->b;
  const int grid = rowgram_grid(ctx->nloc);
  if (G && (size_t)grid * b * b > ctx->slab_elems)
    return fail(ctx, RBL_ERR_INVALID, "internal: row-op slab too small");
  if (ctx->nloc > 0) {
    // without a Gram the grid follows the kernel's occupancy (no partials to count)
    rowgram(ctx->nloc, b, X, C, b, Y, alpha, beta, G ? ctx->d_slab : nullptr, G ? grid : 0, skip,
            ctx->stream, X32, Y32, f64flag, tri && !X32);
    HIPC(hipGetLastError());
  } else if (G) {  // no rows on this rank: its share of the Gram is zero (the all-reduce still runs)
    HIPC(hipMemsetAsync(ctx->d_slab, 0, (size_t)grid * b * b * sizeof(double), ctx->stream));
  }
  if (!G) return RBL_OK;
  reduce_slab(ctx->d_slab, grid, (int64_t)b * b, G, skip, ctx->stream);
  HIPC(hipGetLastError());
  return allreduce(ctx, G, (size_t)b * b);
}

// Gram slab of a run (doubles): the largest Gram is the partial-reorth one, (max_blocks-1)
// panels x 2b per split; also the row ops' partials, the partial-reorth update's local-reorth
// Gram partials and the fp32 Grams.  rbl_start allocates it; the automatic device-block plan
// (RBL_OPT_DEVICE_BLOCKS < 0) budgets it — one formula for both.
size_t gram_slab_elems(const rbl_ctx* ctx, int b, int max_blocks, int basis_bits) {
  size_t slab = 0;
  for (int nW = 1; nW <= std::max(1, max_blocks - 1); ++nW)
    for (int xc : {b, 2 * b}) {
      const size_t sp = (size_t)gram_splits(ctx->nloc, nW, b, xc);
      slab = std::max(slab, sp * nW * b * xc);
    }
  slab = std::max(slab, (size_t)2 * rowgram_grid(ctx->nloc, kRowgramMaxPerCu) * b * b);  // rowop partials (+ cross Gram)
  // the partial-reorth update's local-reorth Gram partials (one b x b per 128-row tile:
  // n_local b^2 / 128 doubles, a quarter of a block at b = 32)
  if (b == 32 && basis_bits == 64 && (ctx->fuse & 2)) {
    const int xg = tsmm44_xg_grid(ctx->nloc);
    slab = std::max(slab, (size_t)(xg + reduce_scratch_splits(xg)) * b * b);
  }
  if (basis_bits == 32)  // fp32 Grams: up to (max_blocks-1) panels x 2b per split
    slab = std::max(slab, (size_t)gram32_splits(ctx->nloc) * std::max(1, max_blocks - 1) * b * 2 * b);
  return slab;
}

bool has_matrix(const rbl_ctx* ctx) { return ctx->d_rowptr || ctx->dense; }

// fp32 basis: the band-tile SpMM and the 3-term update read the fp32 blocks directly
bool direct32_ok(const rbl_ctx* ctx, int b) {
  return !ctx->dense && (ctx->spmm_variant == 0 || ctx->spmm_variant == 4) && (b == 32 || b == 16) &&
         (ctx->bt_ng == 5 || ctx->bt_ng == 9);
}
// the fp64 scratch block of the fp32 path (widened Q_{i-1}, Ritz / get_block widening),
// allocated on first use when the direct path made it unnecessary at rbl_start
int ensure_qm64(rbl_ctx* ctx) {
  if (ctx->d_Qm64) return RBL_OK;
  HIPC(hipMalloc(&ctx->d_Qm64, (std::max<int64_t>(ctx->nloc, 1) + kRowPad) * ctx->b * sizeof(double)));
  return RBL_OK;
}

// The indexed halo serves only the segmented gather's own / halo column tiers (b in {16, 32});
// any other SpMM (another b, a kernel pinned by RBL_OPT_SPMM_KERNEL) reads the range halo,
// which is kept beside it.  The rule depends only on state every rank shares (the collective
// `ghost` decision, b, the option), so all ranks pick the same exchange for a call.
bool use_ghost(const rbl_ctx* ctx, int b) {
  return ctx->ghost && ctx->nranks > 1 && (b == 16 || b == 32) &&
         (ctx->spmm_variant == 0 || ctx->spmm_variant == 5);
}
// rows of the halo buffer for block size b: the ghost slots, or the range [ext_lo, ext_hi)
int64_t qext_rows(const rbl_ctx* ctx, int b) {
  return std::max<int64_t>(use_ghost(ctx, b) ? ctx->n_ghost : ctx->ext_hi - ctx->ext_lo, 1);
}
// grow the halo buffer (zeroed: rows between the received ranges stay finite) for block size b
int ensure_qext(rbl_ctx* ctx, int b, hipStream_t st) {
  const size_t need = (size_t)qext_rows(ctx, b) * b;
  if (ctx->d_qext && ctx->qext_cap >= need) return RBL_OK;
  HIPC(hipStreamSynchronize(ctx->stream));
  hipFree(ctx->d_qext);
  ctx->d_qext = nullptr;
  ctx->qext_cap = 0;
  HIPC(hipMalloc(&ctx->d_qext, need * sizeof(double)));
  HIPC(hipMemsetAsync(ctx->d_qext, 0, need * sizeof(double), st));
  ctx->qext_cap = need;
  return RBL_OK;
}

// U = A Qin (+ U -= Qprev Bi^T when Qprev): the SpMM of RBL_gpu.jl:176-177, or for a dense
// A (RBL_gpu.jl:205 with A::Matrix) the panel GEMM on fp64 MFMA (tsmm44 over the panels of
// the local rows, Q gathered to all n rows by the halo exchange).  Returns the number of
// A_i partials the band kernel formed in `slab` (0: none), or a negative status.
int apply_A(rbl_ctx* ctx, const double* Qin, int64_t off, int b, double* U, const double* Qprev,
            const double* Bi, double* slab, const double* qloc = nullptr,
            const double* lfix_c = nullptr, double* lfix_q = nullptr, int64_t lf_lo = 0,
            int64_t lf_hi = 0, hipEvent_t seg_wait = nullptr) {
  if (ctx->nloc <= 0) return 0;
  if (ctx->csr_dropped && rbl_spmm_kernel_for(ctx, b) != 5)
    return fail(ctx, RBL_ERR_STATE, "the CSR was released (RBL_OPT_KEEP_CSR = 0): only the band-tile "
                                    "SpMM (b in {16, 32}) can run");
  if (!ctx->dense) {
    CsrDev A = csr(ctx);
    // indexed halo: the own-column tier always reads the block the exchange sent from (a rank
    // without nonzeros runs the plain gather, which reads no Q row at all)
    if (!qloc && ctx->ghost_active && ctx->nranks > 1 && rbl_spmm_kernel_for(ctx, b) == 6)
      qloc = ctx->ghost_local;
    if (qloc) {  // own rows from the block itself (halo_exchange without the local copy)
      A.qloc = qloc;
      A.loc_lo = ctx->r0;
      A.loc_hi = ctx->r0 + ctx->nloc;
    }
    A.seg_wait = seg_wait;  // own/halo column tiers: the halo tier waits for the exchange
    int two_wave = 0;
    A.two_wave = &two_wave;
    if (lfix_c) {  // local reorth fused into the SpMM's staging (RBL_OPT_FUSE bit 2)
      A.lfix_c = lfix_c;
      A.lfix_q = lfix_q;
      A.lfix_lo = lf_lo;
      A.lfix_hi = lf_hi;
    }
    const int parts = spmm(A, Qin, off, b, U, Qprev, Bi, ctx->spmm_variant, ctx->stream, slab);
    if (parts < 0) return fail(ctx, RBL_ERR_INVALID, "internal: split-source SpMM needs the band-tile kernel");
    ctx->path_stats[RBL_PATH_SPMM] += 1;
    ctx->path_stats[RBL_PATH_SPMM_TWO_WAVE] += two_wave;
    if (lfix_c) {
      ctx->path_stats[RBL_PATH_SPMM_LOC_FUSED] += 1;
      ctx->path_stats[RBL_PATH_LOCFIX_REST] += 1;
      StageScope t(ctx, RBL_STAGE_LOC_REORTH);
      spmm_bt_locfix_rest(A, lfix_q, Qprev, lfix_c, ctx->stream);
    }
    return parts;
  }
  if (b > ctx->qfull_cols) {  // Q gathered to all n rows, zero-padded to 32 * dense_panels
    hipFree(ctx->d_qfull);
    ctx->d_qfull = nullptr;
    ctx->qfull_cols = 0;
    HIPC(hipMalloc(&ctx->d_qfull, (size_t)ctx->dense_panels * 32 * b * sizeof(double)));
    HIPC(hipMemsetAsync(ctx->d_qfull, 0, (size_t)ctx->dense_panels * 32 * b * sizeof(double), ctx->stream));
    ctx->qfull_cols = b;
  }
  HIPC(hipMemcpyAsync(ctx->d_qfull, Qin + (0 - off) * b, ctx->n * b * sizeof(double),
                      hipMemcpyDeviceToDevice, ctx->stream));
  PanelRun X;
  X.base = ctx->d_dense;
  X.stride = ctx->nloc * 32;
  X.w = 32;
  X.count = (int)ctx->dense_panels;
  CHK(tsmm_checked(ctx, X, ctx->d_qfull, b, pan1(U, b), 1.0, 0.0, nullptr));
  if (Qprev) {
    transpose_small(Bi, smallp(ctx, S_BT), b, ctx->stream);
    CHK(tsmm_checked(ctx, run1(Qprev, b), smallp(ctx, S_BT), b, pan1(U, b), -1.0, 1.0, nullptr));
  }
  return 0;
}

// X -= l (l^T X) for every locked vector l in lock order (restarted.jl:1-21,
// restart_reorth_gpu!: one projection per locked vector, MGS over them).
int lock_reorth(rbl_ctx* ctx, double* X) {
  const int b = ctx->b;
  for (int j = 0; j < ctx->nlock; ++j) {
    const double* l = ctx->d_lock + (int64_t)j * ctx->nloc;
    CHK(gram(ctx, run1(l, 1), pan1(X, b), ctx->d_C, nullptr));
    CHK(tsmm_checked(ctx, run1(l, 1), ctx->d_C, b, pan1(X, b), -1.0, 1.0, nullptr));
  }
  return RBL_OK;
}

// Reorth of the pair (Q_i, Q_{i-1}) = slots (i-1, i-2) of the fp64 basis:
//   flags bit 1: against the locked vectors, Q_{i-1} then Q_i (restarted.jl:54-55);
//   flags bit 0: against Q_1..Q_{i-2} (RBL_gpu.jl:59-81; block CGS, or the reference's
//                ascending-j block MGS with RBL_OPT_REORTH_ORDER = 1).
// i == 1 with bit 1: Q_1 against the locked vectors (restarted.jl:41).
int reorth_pair(rbl_ctx* ctx, int i, int flags) {
  const int b = ctx->b;
  double* Qi = slotp(ctx, i - 1);
  double* Qm = i >= 2 ? slotp(ctx, i - 2) : nullptr;
  if ((flags & 2) && ctx->nlock > 0) {
    StageScope t(ctx, RBL_STAGE_PART_REORTH);
    if (Qm) CHK(lock_reorth(ctx, Qm));
    CHK(lock_reorth(ctx, Qi));
  }
  if ((flags & 1) && i >= 3) {
    StageScope t(ctx, RBL_STAGE_PART_REORTH);
    const int nW = i - 2;
    const int nres = std::min(nW, ctx->resident);  // HBM-resident part of W
    // the last update of the pair also forms this step's local-reorth Gram Q_{i-1}^T Q_i
    // (RBL_OPT_FUSE bit 1; the update's 64-column fast path: b = 32)
    // (the same decision on every rank: the all-reduce below pairs up; a rank where the fast
    // path does not apply — too few rows, slab too small — forms its share with the Gram kernel)
    const bool xg = (ctx->fuse & 2) && b == 32;
    const int xg_parts = tsmm44_xg_grid(ctx->nloc);
    const bool xslab_ok = (size_t)(xg_parts + reduce_scratch_splits(xg_parts)) * b * b <= ctx->slab_elems;
    int xgrid = 0;
    auto update = [&](const PanelRun& W, bool last) -> int {
      const bool here = xg && last && xslab_ok;
      return tsmm_checked(ctx, W, ctx->d_C, 2 * b, pan2(Qi, Qm, b), -1.0, 1.0, nullptr,
                          here ? ctx->d_slab : nullptr, here ? &xgrid : nullptr);
    };
    if (ctx->reorth_order == 0) {  // block CGS: one Gram over every resident j, one update
      PanelRun W;
      W.base = slotp(ctx, 0);
      W.stride = ctx->slot;
      W.count = nres;
      W.w = b;
      CHK(gram(ctx, W, pan2(Qi, Qm, b), ctx->d_C, nullptr));
      CHK(update(W, nres == nW));
    } else {  // ascending-j block MGS, exactly the reference order
      for (int j = 0; j < nres; ++j) {
        const PanelRun W = run1(slotp(ctx, j), b);
        CHK(gram(ctx, W, pan2(Qi, Qm, b), ctx->d_C, nullptr));
        CHK(update(W, j == nW - 1));
      }
    }
    // spilled blocks (host, final): streamed back one at a time, ascending j, each applied
    // as soon as it lands — hybrid_part_reorth!'s `copyto!(Qgj, Q[j]); part_reorth_gpu!`
    // (RBL_gpu.jl:65-68)
    for (int j = nres; j < nW; ++j) {
      int st = 0;
      const double* Wj = block_dev(ctx, j, i, &st);
      if (st) return fail(ctx, st, "partial reorth: H2D of a spilled block failed");
      CHK(gram(ctx, run1(Wj, b), pan2(Qi, Qm, b), ctx->d_C, nullptr));
      CHK(update(run1(Wj, b), j == nW - 1));
    }
    if (xg) {  // the partials of the last update (its Gram slab was reduced before it)
      if (xgrid > 0) {
        reduce_slab_many(ctx->d_slab, xgrid, (int64_t)b * b, smallp(ctx, S_CLOC), ctx->stream);
      } else if (ctx->nloc > 0) {
        const int sp = gram_splits(ctx->nloc, 1, b, b);
        gram_partial(ctx->nloc, run1(Qm, b), pan1(Qi, b), ctx->d_slab, sp, nullptr, ctx->stream);
        reduce_slab(ctx->d_slab, sp, (int64_t)b * b, smallp(ctx, S_CLOC), nullptr, ctx->stream);
      } else {
        HIPC(hipMemsetAsync(smallp(ctx, S_CLOC), 0, (size_t)b * b * sizeof(double), ctx->stream));
      }
      HIPC(hipGetLastError());
      CHK(allreduce(ctx, smallp(ctx, S_CLOC), (size_t)b * b));
      ctx->cloc_step = i;
      ctx->cloc_final = true;
    }
  }
  return RBL_OK;
}

// Y = [Q_1 .. Q_nblocks] S_dev (S_dev device row-major (nblocks*b) x kcols): one run over the
// HBM-resident blocks, then every other block (streamed from the host when spilled)
int combine_blocks(rbl_ctx* ctx, int nblocks, int kcols, const double* d_S, double* Y) {
  const int b = ctx->b;
  const int nres = std::min(nblocks, ctx->resident);
  PanelRun X;
  X.base = slotp(ctx, 0);
  X.stride = ctx->slot;
  X.count = nres;
  X.w = b;
  CHK(tsmm_checked(ctx, X, d_S, kcols, pan1(Y, kcols), 1.0, 0.0, nullptr));
  for (int j = nres; j < nblocks; ++j) {
    int st = 0;
    const double* Qj = block_dev(ctx, j, ctx->nblocks, &st);
    if (st) return fail(ctx, st, "Ritz: H2D of a spilled block failed");
    CHK(tsmm_checked(ctx, run1(Qj, b), d_S + (int64_t)j * b * kcols, kcols, pan1(Y, kcols), 1.0,
                     1.0, nullptr));
  }
  return RBL_OK;
}

// Y (n_local x kcols, row-major) = [Q_1 .. Q_nblocks] S with S host (nblocks*b) x kcols
// column-major — the Ritz combination of RBL.jl:61-71 / RBL_gpu.jl:106-132 (fp64 basis).
int basis_combine(rbl_ctx* ctx, int nblocks, int kcols, const double* S, double* Y) {
  const int b = ctx->b;
  const int64_t rows = (int64_t)nblocks * b;
  double *d_Scm = nullptr, *d_S = nullptr;
  HIPC(hipMalloc(&d_Scm, rows * kcols * sizeof(double)));
  HIPC(hipMalloc(&d_S, rows * kcols * sizeof(double)));
  HIPC(hipMemcpyAsync(d_Scm, S, rows * kcols * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  colmajor_to_rowmajor(d_Scm, rows, kcols, d_S, ctx->stream);
  const int st = combine_blocks(ctx, nblocks, kcols, d_S, Y);
  HIPC(hipStreamSynchronize(ctx->stream));
  hipFree(d_S);
  hipFree(d_Scm);
  return st;
}

// Y = [Q_1 .. Q_nblocks] S_dev over the fp32 basis, widened on load, V and S fp64 (P3: fp64
// Ritz): one launch over the resident blocks when the fp32-input tsmm44 applies, else each
// block widened into a scratch block and accumulated; spilled blocks stream from the host
int combine_blocks32(rbl_ctx* ctx, int nblocks, int kcols, const double* d_S, double* Y) {
  const int b = ctx->b;
  if (ctx->nloc <= 0) return RBL_OK;
  const int nres = std::min(nblocks, ctx->resident);
  int j0 = 0;
  if (tsmm44_ok(b, kcols, kcols) && nres > 0) {
    PanelRun X;
    X.base32 = slotp32(ctx, 0);
    X.stride = ctx->slot;
    X.count = nres;
    X.w = b;
    tsmm44_f32x(ctx->nloc, X, d_S, kcols, pan1(Y, kcols), 1.0, 0.0, ctx->stream);
    HIPC(hipGetLastError());
    j0 = nres;
  }
  if (j0 < nblocks) CHK(ensure_qm64(ctx));
  for (int j = j0; j < nblocks; ++j) {
    int st = 0;
    const float* Qj = block_dev32(ctx, j, ctx->nblocks, &st);
    if (st) return fail(ctx, st, "Ritz: H2D of a spilled block failed");
    cvt_f32_to_f64(Qj, ctx->d_Qm64, ctx->nloc * b, ctx->stream);
    CHK(tsmm_checked(ctx, run1(ctx->d_Qm64, b), d_S + (int64_t)j * b * kcols, kcols, pan1(Y, kcols),
                     1.0, j == 0 ? 0.0 : 1.0, nullptr));
  }
  return RBL_OK;
}

// fp32 basis: Gram C = W^T [X0, X1] over all ranks (fp32 MFMA per split, fp64 sum), C fp64
// [nW*b][xcount*b] — the FLOAT `temp` of RBL_gpu.jl:33,39,87 (rounded to f32 where applied).
int gram32(rbl_ctx* ctx, const float* Wb, int nW, const float* X0, const float* X1, int xcount,
           double* C) {
  const int b = ctx->b;
  const int splits = gram32_splits(ctx->nloc);
  const int64_t len = (int64_t)nW * b * xcount * b;
  if ((size_t)splits * len > ctx->slab_elems)
    return fail(ctx, RBL_ERR_INVALID, "internal: Gram slab too small (fp32)");
  if (ctx->nloc > 0) {
    gram32_partial(ctx->nloc, Wb, ctx->slot, nW, b, X0, X1, xcount, ctx->d_slab, splits, ctx->stream);
    reduce_slab(ctx->d_slab, splits, len, C, nullptr, ctx->stream);
  } else {
    HIPC(hipMemsetAsync(C, 0, len * sizeof(double), ctx->stream));
  }
  HIPC(hipGetLastError());
  return allreduce(ctx, C, (size_t)len);
}
// fp32 basis: [Y0, Y1] -= X C (X: nX fp32 slots from Xb), RBL_gpu.jl:34,40,88 in FLOAT.
int upd32(rbl_ctx* ctx, const float* Xb, int nX, const double* C, int ldc, float* Y0, float* Y1,
          int ycount) {
  if (ctx->nloc <= 0) return RBL_OK;
  tsmm32(ctx->nloc, Xb, ctx->slot, nX, ctx->b, C, ldc, Y0, Y1, ycount, -1.f, 1.f, ctx->stream);
  HIPC(hipGetLastError());
  return RBL_OK;
}

// Fused row op in one of the CholQR forms (RowOpArgs: mode 1 Gram only, mode 2 two-stage
// apply, Z for a cross Gram).  G: the Gram (mode 1) over all ranks; Gx: Z^T Y over all ranks
// (reduced only when reduce_x).
int rowop_ex(rbl_ctx* ctx, RowOpArgs a, double* G, double* Gx, bool reduce_x, bool comm_x = true) {
  const int b = ctx->b;
  const int gmax = rowgram_grid(ctx->nloc, kRowgramMaxPerCu);
  if ((size_t)2 * gmax * b * b > ctx->slab_elems)
    return fail(ctx, RBL_ERR_INVALID, "internal: row-op slab too small");
  if (G) a.slab = ctx->d_slab;
  if (a.Z) a.slab2 = ctx->d_slab + (size_t)gmax * b * b;
  // the cross-Gram launches (pass 2, and pass 3 when it runs) share one grid: the reduce
  // after pass 3 does not know which of them wrote the partials last
  const int xgrid = rowgram_grid(ctx->nloc, 2);
  int grid = a.Z ? xgrid : 0;
  a.grid_out = &grid;
  if (ctx->nloc > 0) {
    if (!rowgram_ex(ctx->nloc, b, a, grid, ctx->stream))
      return fail(ctx, RBL_ERR_INVALID, "internal: unsupported fused row-op form");
  } else {  // no rows on this rank: zero partials (the all-reduces still run on every rank)
    grid = 1;
    if (G) HIPC(hipMemsetAsync(a.slab, 0, (size_t)b * b * sizeof(double), ctx->stream));
    if (a.Z && a.skip == nullptr)
      HIPC(hipMemsetAsync(a.slab2, 0, (size_t)xgrid * b * b * sizeof(double), ctx->stream));
  }
  HIPC(hipGetLastError());
  if (G) {
    reduce_slab(ctx->d_slab, grid, (int64_t)b * b, G, a.skip, ctx->stream);
    CHK(allreduce(ctx, G, (size_t)b * b));
  }
  if (Gx && reduce_x) {
    reduce_slab(ctx->d_slab + (size_t)gmax * b * b, xgrid, (int64_t)b * b, Gx, nullptr, ctx->stream);
    if (comm_x) CHK(allreduce(ctx, Gx, (size_t)b * b));
  }
  return RBL_OK;
}

// Tall-skinny QR of U (n_local x b) into Qout; B = R (b x b, upper, row-major) in S_RTOT.
// Shifted CholQR2 (+ a third pass after a shifted first pass).  `g1_ready`: S_G already holds
// U^T U (the fused 3-term update computed it); each apply computes the next pass's Gram in the
// same pass over the rows when b allows (rowop).
// Qout32 (fp32 basis): the final Q goes to Qout32 rounded to fp32 (Qout then holds only a
// pass-2 intermediate when the shifted pass 3 runs).
// Zloc (fp64 basis, RBL_OPT_FUSE bit 1): also form Zloc^T Q into S_CLOC — the next step's
// local-reorth coefficient (Zloc = Q_i, Q = Q_{i+1}).
int tsqr(rbl_ctx* ctx, const double* U, double* Qout, bool g1_ready = false, float* Qout32 = nullptr,
         const double* Zloc = nullptr) {
  StageScope t(ctx, RBL_STAGE_QR);
  ctx->flags_clean = false;  // the flags below start from zero only after a memset or k_stash
  const int b = ctx->b;
  int* need3 = ctx->d_flags;      // [need3, skip3]
  int* status = ctx->d_flags + 2; // [breakdown, shifted count]
  double* G = smallp(ctx, S_G);
  const int* skip3 = need3 + 1;
  const bool fused = rowgram_ok(b);
  // Qout = Qout R^-1: in place while one wave owns whole rows (tsmm: b <= 64), else through
  // the scratch block T
  auto apply_inplace = [&](const int* skip) -> int {
    if (b <= 64)
      return tsmm_checked(ctx, run1(Qout, b), smallp(ctx, S_RINV), b, pan1(Qout, b), 1.0, 0.0, skip);
    CHK(tsmm_checked(ctx, run1(Qout, b), smallp(ctx, S_RINV), b, pan1(ctx->d_T, b), 1.0, 0.0, skip));
    copy_small(ctx->d_T, Qout, ctx->nloc * b, ctx->stream, skip);
    return RBL_OK;
  };
  // pass 1 (shift decided on device); the 3-pass form keeps R1^-1 (S_RINV1) for its last pass
  const bool three = fused && (ctx->fuse & 1);
  if (!g1_ready) CHK(gram(ctx, run1(U, b), pan1(U, b), G, nullptr));
  chol_step(G, b, ctx->n, 0, smallp(ctx, S_R), smallp(ctx, three ? S_RINV1 : S_RINV), smallp(ctx, S_RTOT),
            need3, status, nullptr, ctx->stream, smallp(ctx, S_CHS0));
  if (three) {
    // 3 passes: G2 = Gram of Q1 = U R1^-1 without storing Q1; then Q = (U R1^-1) R2^-1 in
    // one pass (Q1 recomputed bit for bit) — the same bits as the 4-pass form below
    RowOpArgs a1;
    a1.X = U;
    a1.C = smallp(ctx, S_RINV1);
    a1.ldc = b;
    a1.mode = 1;
    a1.tri = true;  // R^-1
    CHK(rowop_ex(ctx, a1, G, nullptr, false));
    chol_step(G, b, ctx->n, 1, smallp(ctx, S_R), smallp(ctx, S_RINV), smallp(ctx, S_RTOT), need3,
              status, nullptr, ctx->stream, smallp(ctx, S_CHS0));
    RowOpArgs a2;
    a2.X = U;
    a2.C = smallp(ctx, S_RINV1);
    a2.C2 = smallp(ctx, S_RINV);
    a2.ldc = b;
    a2.tri = true;  // R1^-1, R2^-1
    a2.Y = Qout;
    a2.Y32 = Qout32;
    a2.f64flag = Qout32 ? need3 : nullptr;
    a2.Z = Zloc;
    a2.mode = 2;
    // Zloc: this rank's share of Zloc^T Q2 now, all-reduced below with the pass-3 Gram
    CHK(rowop_ex(ctx, a2, nullptr, Zloc ? smallp(ctx, S_CLOC) : nullptr, Zloc != nullptr, false));
    // pass 3 only after a shifted first pass (device flag; kernels early-exit otherwise).  Its
    // Gram's all-reduce runs either way (the host does not know the flag) and carries Zloc^T Q2
    // in the same call (S_CLOC follows S_G)
    CHK(gram(ctx, run1(Qout, b), pan1(Qout, b), G, skip3, Zloc == nullptr));
    if (Zloc) CHK(allreduce(ctx, G, (size_t)2 * b * b));
    chol_step(G, b, ctx->n, 1, smallp(ctx, S_R), smallp(ctx, S_RINV), smallp(ctx, S_RTOT), need3,
              status, skip3, ctx->stream, smallp(ctx, S_CHS0));
    RowOpArgs a3;
    a3.X = Qout;
    a3.C = smallp(ctx, S_RINV);
    a3.ldc = b;
    a3.tri = true;
    a3.Y = Qout;
    a3.skip = skip3;
    a3.Y32 = Qout32;
    a3.mode = 0;
    CHK(rowop_ex(ctx, a3, nullptr, nullptr, false));
    // after a third pass Q3 = Q2 R3^-1: Zloc^T Q3 = (Zloc^T Q2) R3^-1 (no-op unless it ran)
    if (Zloc) cloc_rinv(smallp(ctx, S_CLOC), smallp(ctx, S_RINV), b, skip3, ctx->stream);
    HIPC(hipGetLastError());
    return RBL_OK;
  }
  if (Zloc) return fail(ctx, RBL_ERR_INVALID, "internal: local-reorth Gram fusion needs the 3-pass QR");
  if (fused) {
    CHK(rowop(ctx, U, smallp(ctx, S_RINV), Qout, 1.0, 0.0, G, nullptr, nullptr, nullptr, nullptr, true));
  } else {
    CHK(tsmm_checked(ctx, run1(U, b), smallp(ctx, S_RINV), b, pan1(Qout, b), 1.0, 0.0, nullptr));
    CHK(gram(ctx, run1(Qout, b), pan1(Qout, b), G, nullptr));
  }
  // pass 2
  chol_step(G, b, ctx->n, 1, smallp(ctx, S_R), smallp(ctx, S_RINV), smallp(ctx, S_RTOT), need3,
            status, nullptr, ctx->stream, smallp(ctx, S_CHS0));
  if (fused) {  // in place; the Gram feeds pass 3 when a shifted first pass asked for it
    // (fp32 basis: the result goes straight to Qout32 unless pass 3 follows)
    CHK(rowop(ctx, Qout, smallp(ctx, S_RINV), Qout, 1.0, 0.0, G, nullptr, nullptr, Qout32,
              Qout32 ? need3 : nullptr, true));
  } else {
    CHK(apply_inplace(nullptr));
    CHK(gram(ctx, run1(Qout, b), pan1(Qout, b), G, skip3));
  }
  // pass 3 only after a shifted first pass (device flag; kernels early-exit otherwise)
  chol_step(G, b, ctx->n, 1, smallp(ctx, S_R), smallp(ctx, S_RINV), smallp(ctx, S_RTOT), need3,
            status, skip3, ctx->stream, smallp(ctx, S_CHS0));
  if (fused) {
    CHK(rowop(ctx, Qout, smallp(ctx, S_RINV), Qout, 1.0, 0.0, nullptr, skip3, nullptr, Qout32,
              nullptr, true));
  } else {
    CHK(apply_inplace(skip3));
    if (Qout32) cvt_f64_to_f32(Qout, Qout32, ctx->nloc * b, ctx->stream);
  }
  HIPC(hipGetLastError());
  return RBL_OK;
}

// Bring Q (n_local x b, local rows) into the halo-extended buffer for SpMM.  copy_local
// false: only the neighbours' rows land there (the band-tile SpMM reads the own rows from Q
// itself, CsrDev::qloc), saving a read + write of the whole local block per step.
int halo_exchange(rbl_ctx* ctx, const double* Q, const double** Qin, int64_t* off,
                  bool copy_local = true, hipStream_t st = nullptr) {
  if (ctx->nranks == 1) {
    *Qin = Q;
    *off = 0;
    return RBL_OK;
  }
  if (!st) st = ctx->stream;
  StageScope t(ctx, RBL_STAGE_COMM, st);
  const int b = ctx->b;
  CHK(ensure_qext(ctx, b, st));
  double* ext = ctx->d_qext;
  ctx->ghost_active = use_ghost(ctx, b);
  if (ctx->ghost_active) {  // indexed halo: pack the asked-for rows, receive into the ghost slots
    gather_rows(Q, ctx->d_send_idx, ctx->n_send, b, ctx->d_sendbuf, st);
    HIPC(hipGetLastError());
    std::vector<Comm::Xfer> x(ctx->nranks);
    for (int q = 0; q < ctx->nranks; ++q) {
      if (q == ctx->rank) continue;
      x[q].send = ctx->d_sendbuf + ctx->send_off[q] * b;
      x[q].nsend = (size_t)ctx->send_cnt[q] * b;
      x[q].recv = ext + ctx->ghost_off[q] * b;
      x[q].nrecv = (size_t)ctx->ghost_cnt[q] * b;
    }
    CHK(exchange(ctx, x, st));
    ctx->ghost_local = Q;
    *Qin = ext;
    *off = 0;
    return RBL_OK;
  }
  if (copy_local)
    HIPC(hipMemcpyAsync(ext + (ctx->r0 - ctx->ext_lo) * b, Q, ctx->nloc * b * sizeof(double),
                        hipMemcpyDeviceToDevice, st));
  std::vector<Comm::Xfer> x(ctx->nranks);
  for (int q = 0; q < ctx->nranks; ++q) {
    if (q == ctx->rank) continue;
    const int64_t gl = ctx->give_lo[q], gh = ctx->give_hi[q];
    if (gh > gl) {
      x[q].send = Q + (gl - ctx->r0) * b;
      x[q].nsend = (size_t)(gh - gl) * b;
    }
    const int64_t nl = ctx->need_lo[q], nh = ctx->need_hi[q];
    if (nh > nl) {
      x[q].recv = ext + (nl - ctx->ext_lo) * b;
      x[q].nrecv = (size_t)(nh - nl) * b;
    }
  }
  CHK(exchange(ctx, x, st));
  *Qin = ext;
  *off = ctx->ext_lo;
  return RBL_OK;
}

// fp32 halo exchange (the fp32 basis read directly by the band-tile SpMM): the same row
// ranges as halo_exchange, fp32 rows moved as byte-identical pairs (b is even)
int halo_exchange32(rbl_ctx* ctx, const float* Q, const float** Qin, int64_t* off,
                    bool copy_local = true) {
  if (ctx->nranks == 1) {
    *Qin = Q;
    *off = 0;
    return RBL_OK;
  }
  StageScope t(ctx, RBL_STAGE_COMM);
  const int b = ctx->b;
  float* ext = reinterpret_cast<float*>(ctx->d_qext);
  if (copy_local)
    HIPC(hipMemcpyAsync(ext + (ctx->r0 - ctx->ext_lo) * b, Q, ctx->nloc * b * sizeof(float),
                        hipMemcpyDeviceToDevice, ctx->stream));
  std::vector<Comm::Xfer> x(ctx->nranks);
  for (int q = 0; q < ctx->nranks; ++q) {
    if (q == ctx->rank) continue;
    const int64_t gl = ctx->give_lo[q], gh = ctx->give_hi[q];
    if (gh > gl) {
      x[q].send = reinterpret_cast<const double*>(Q + (gl - ctx->r0) * b);
      x[q].nsend = (size_t)(gh - gl) * b / 2;
    }
    const int64_t nl = ctx->need_lo[q], nh = ctx->need_hi[q];
    if (nh > nl) {
      x[q].recv = reinterpret_cast<double*>(ext + (nl - ctx->ext_lo) * b);
      x[q].nrecv = (size_t)(nh - nl) * b / 2;
    }
  }
  CHK(exchange(ctx, x, ctx->stream));
  *Qin = ext;
  *off = ctx->ext_lo;
  return RBL_OK;
}

// A/B switches of the variants build (tools/build_variant.sh with -DRBL_VARIANTS): the plain
// D2H copy instead of the staged one (RBL_D2H_DIRECT), the one-pass Ritz (RBL_RITZ_SERIAL)
#ifdef RBL_VARIANTS
bool d2h_direct() { return std::getenv("RBL_D2H_DIRECT") != nullptr; }
bool ritz_serial() { return std::getenv("RBL_RITZ_SERIAL") != nullptr; }
#else
constexpr bool d2h_direct() { return false; }
constexpr bool ritz_serial() { return false; }
#endif

// one step's record in the async stash: A_i, R_tot (b x b each) and 4 int flags (2 doubles)
size_t stash_rec(int b) { return (size_t)2 * b * b + 2; }
// The staged D2H of the Ritz vectors (d2h_staged): two pinned 64 MiB slots and their events,
// kept for the context's life.  Pinning them costs ~20-30 ms, so rbl_start allocates them with
// the run's buffers when a Ritz result will take the staged path (one basis block >= 256 MiB),
// instead of the first rbl_ritz of the context paying it (profiles/r05_ttk_probe.log).
constexpr size_t kD2HPiece = size_t(64) << 20;
int ensure_d2h_slots(rbl_ctx* ctx) {
  for (int s = 0; s < 2; ++s) {
    if (!ctx->h_d2h[s]) HIPC(hipHostMalloc(&ctx->h_d2h[s], kD2HPiece, hipHostMallocDefault));
    if (!ctx->ev_d2h_slot[s]) HIPC(hipEventCreateWithFlags(&ctx->ev_d2h_slot[s], hipEventDisableTiming));
  }
  return RBL_OK;
}

// The pipelined Ritz vectors' side stream and events (ritz_pipelined).  A stream's first launch
// costs ~25 ms (measured: the first pipelined rbl_ritz of a process took 60 ms against 31 ms for
// the next), so rbl_start creates them with the staging slots and runs one empty launch on the
// stream, instead of a time-to-k's Ritz step paying it.
int ensure_ritz_stream(rbl_ctx* ctx) {
  if (!ctx->rstream) {
    HIPC(hipStreamCreateWithFlags(&ctx->rstream, hipStreamNonBlocking));
    copy_small(ctx->d_small, ctx->d_small, 0, ctx->rstream);
    HIPC(hipGetLastError());
    HIPC(hipStreamSynchronize(ctx->rstream));
  }
  for (hipEvent_t& e : ctx->ev_ritz)
    if (!e) HIPC(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  return RBL_OK;
}

// ---- the pushed half of the split halo (prepare_push) ----
bool push_on(const rbl_ctx* ctx) { return ctx->push && ctx->ghost_active && ctx->nranks > 1; }

int ensure_push(rbl_ctx* ctx, int b) {
  const size_t need = (size_t)std::max<int64_t>(std::max(ctx->push_rows, ctx->n_send), 1) * b;
  if (ctx->d_pushbuf && ctx->push_cap >= need) return RBL_OK;
  HIPC(hipStreamSynchronize(ctx->stream));
  if (ctx->hstream) HIPC(hipStreamSynchronize(ctx->hstream));
  hipFree(ctx->d_pushbuf); ctx->d_pushbuf = nullptr;
  hipFree(ctx->d_precv); ctx->d_precv = nullptr;
  ctx->push_cap = 0;
  HIPC(hipMalloc(&ctx->d_pushbuf, need * sizeof(double)));
  HIPC(hipMalloc(&ctx->d_precv, need * sizeof(double)));
  ctx->push_cap = need;
  return RBL_OK;
}

// partial rows for the peers' ghost slots from the own rows of Q (n_local x b)
int push_products(rbl_ctx* ctx, const double* Q, int b, hipStream_t st) {
  StageScope t(ctx, RBL_STAGE_AQ, st);
  CHK(ensure_push(ctx, b));
  const auto& P = ctx->push_tier;
  CsrDev::Tier T;
  T.rowptr = P.rowptr;
  T.col = P.col;
  T.val = P.val;
  T.ntasks = P.ntasks;
  T.nlong = P.nlong;
  T.trow = P.trow;
  T.tinfo = P.tinfo;
  T.slot_k0 = P.slot_k0;
  T.lrow = P.lrow;
  T.lslot = P.lslot;
  T.scratch = P.scratch;
  spmm_seg_tier(T, Q, ctx->r0, b, ctx->d_pushbuf, st);
  HIPC(hipGetLastError());
  return RBL_OK;
}

// partials out to the owners of the ghost slots, in from the peers for the rows they asked for
// (the reverse of halo_exchange's directions and counts)
int push_exchange(rbl_ctx* ctx, int b, hipStream_t st) {
  StageScope t(ctx, RBL_STAGE_COMM, st);
  std::vector<Comm::Xfer> x(ctx->nranks);
  for (int q = 0; q < ctx->nranks; ++q) {
    if (q == ctx->rank) continue;
    x[q].send = ctx->d_pushbuf + ctx->ghost_off[q] * b;
    x[q].nsend = (size_t)ctx->ghost_cnt[q] * b;
    x[q].recv = ctx->d_precv + ctx->send_off[q] * b;
    x[q].nrecv = (size_t)ctx->send_cnt[q] * b;
  }
  CHK(exchange(ctx, x, st));
  return RBL_OK;
}

int push_finish(rbl_ctx* ctx, double* U, int b, hipStream_t st) {
  StageScope t(ctx, RBL_STAGE_AQ, st);
  push_add(ctx->d_ps_rows, ctx->d_ps_ptr, ctx->d_ps_slot, ctx->n_ps_rows, ctx->d_precv, b, U, st);
  HIPC(hipGetLastError());
  return RBL_OK;
}

// the whole pushed half on one stream, after apply_A: products, exchange, add
int push_halo(rbl_ctx* ctx, const double* Q, int b, double* U) {
  if (!push_on(ctx)) return RBL_OK;
  CHK(push_products(ctx, Q, b, ctx->stream));
  CHK(push_exchange(ctx, b, ctx->stream));
  return push_finish(ctx, U, b, ctx->stream);
}

void free_run(rbl_ctx* ctx) {
  if (ctx->cstream) hipStreamSynchronize(ctx->cstream);
  hipFree(ctx->d_basis); ctx->d_basis = nullptr;
  for (void* h : ctx->h_spill)
    if (h) hipHostFree(h);
  ctx->h_spill.clear();
  hipFree(ctx->d_stage); ctx->d_stage = nullptr;
  ctx->resident = INT32_MAX;
  ctx->d2h_pending[0] = ctx->d2h_pending[1] = false;
  hipFree(ctx->d_basis32); ctx->d_basis32 = nullptr;
  hipFree(ctx->d_stage32); ctx->d_stage32 = nullptr;
  hipFree(ctx->d_Qi64); ctx->d_Qi64 = nullptr;
  hipFree(ctx->d_Qm64); ctx->d_Qm64 = nullptr;
  ctx->basis_bits = 64;
  hipFree(ctx->d_U); ctx->d_U = nullptr;
  hipFree(ctx->d_T); ctx->d_T = nullptr;
  hipFree(ctx->d_qext); ctx->d_qext = nullptr; ctx->qext_cap = 0;
  hipFree(ctx->d_sendbuf); ctx->d_sendbuf = nullptr;
  if (ctx->hstream) hipStreamSynchronize(ctx->hstream);
  hipFree(ctx->d_pushbuf); ctx->d_pushbuf = nullptr;
  hipFree(ctx->d_precv); ctx->d_precv = nullptr;
  ctx->push_cap = 0;
  hipFree(ctx->d_slab); ctx->d_slab = nullptr;
  hipFree(ctx->d_C); ctx->d_C = nullptr;
  hipFree(ctx->d_small); ctx->d_small = nullptr;
  hipFree(ctx->d_flags); ctx->d_flags = nullptr;
  hipFree(ctx->d_lock); ctx->d_lock = nullptr;
  ctx->nlock = ctx->lock_cap = 0;
  if (ctx->h_pin) hipHostFree(ctx->h_pin);
  ctx->h_pin = nullptr;
  if (ctx->h_hist) hipHostFree(ctx->h_hist);
  ctx->h_hist = nullptr;
  hipFree(ctx->d_stash);
  ctx->d_stash = nullptr;
  ctx->dv_pin = ctx->dv_hist = nullptr;
  ctx->nblocks = 0;
  ctx->b = 0;
  ctx->have_bprev = false;
}

void free_matrix(rbl_ctx* ctx) {
  hipFree(ctx->d_rowptr); ctx->d_rowptr = nullptr;
  hipFree(ctx->d_col); ctx->d_col = nullptr;
  hipFree(ctx->d_val); ctx->d_val = nullptr;
  hipFree(ctx->d_tcmin); ctx->d_tcmin = nullptr;
  hipFree(ctx->d_tcmax); ctx->d_tcmax = nullptr;
  hipFree(ctx->d_tinfo); ctx->d_tinfo = nullptr;
  free_panels(ctx);
  hipFree(ctx->d_bpos); ctx->d_bpos = nullptr;
  hipFree(ctx->d_bt); ctx->d_bt = nullptr;
  hipFree(ctx->d_bth); ctx->d_bth = nullptr;
  hipFree(ctx->d_bte); ctx->d_bte = nullptr;
  hipFree(ctx->d_btp_hdr); ctx->d_btp_hdr = nullptr;
  hipFree(ctx->d_btp_val); ctx->d_btp_val = nullptr;
  hipFree(ctx->d_zrow); ctx->d_zrow = nullptr;
  ctx->bt_ng = 0;
  hipFree(ctx->d_seg_trow); ctx->d_seg_trow = nullptr;
  hipFree(ctx->d_seg_tinfo); ctx->d_seg_tinfo = nullptr;
  hipFree(ctx->d_seg_slot_k0); ctx->d_seg_slot_k0 = nullptr;
  hipFree(ctx->d_seg_lrow); ctx->d_seg_lrow = nullptr;
  hipFree(ctx->d_seg_lslot); ctx->d_seg_lslot = nullptr;
  hipFree(ctx->d_seg_scratch); ctx->d_seg_scratch = nullptr;
  ctx->seg_ntasks = ctx->seg_nlong = 0;
  free_tiers(ctx);
  hipFree(ctx->d_dense); ctx->d_dense = nullptr;
  hipFree(ctx->d_qfull); ctx->d_qfull = nullptr; ctx->qfull_cols = 0;
  ctx->dense = false;
  ctx->dense_panels = 0;
  ctx->n = ctx->nloc = ctx->nnz = 0;
  ctx->ntiles = ctx->tiles_per_wg = 0;
  ctx->window_ok16 = ctx->window_ok32 = false;
  ctx->band_ok16 = ctx->band_ok32 = false;
  ctx->csr_dropped = false;
  ctx->relabeled = false;
}

// Exchange halo needs among ranks and size the extended buffer.
int setup_halo(rbl_ctx* ctx) {
  const int P = ctx->nranks;
  ctx->give_lo.assign(P, 0);
  ctx->give_hi.assign(P, 0);
  ctx->ext_lo = ctx->r0;
  ctx->ext_hi = ctx->r1;
  if (P == 1) return RBL_OK;
  for (int q = 0; q < P; ++q) {
    if (q == ctx->rank || ctx->need_hi[q] <= ctx->need_lo[q]) continue;
    ctx->ext_lo = std::min(ctx->ext_lo, ctx->need_lo[q]);
    ctx->ext_hi = std::max(ctx->ext_hi, ctx->need_hi[q]);
  }
  // all-gather the (lo,hi) need tables: row p of the table = what rank p needs from each q
  std::vector<int64_t> mine(2 * P);
  for (int q = 0; q < P; ++q) {
    mine[2 * q] = ctx->need_lo[q];
    mine[2 * q + 1] = ctx->need_hi[q];
  }
  std::vector<int64_t> all(2 * P * P);
  COMMC(ctx->comm->allgather_host(mine.data(), all.data(), 2 * P, ctx->stream, &ctx->err));
  for (int p = 0; p < P; ++p) {
    if (p == ctx->rank) continue;
    ctx->give_lo[p] = all[(size_t)p * 2 * P + 2 * ctx->rank];
    ctx->give_hi[p] = all[(size_t)p * 2 * P + 2 * ctx->rank + 1];
  }
  return RBL_OK;
}

// Upload a local CSR (0-based rowptr relative to the slice, global 0-based int64 columns).
int upload_csr(rbl_ctx* ctx, int64_t n, int64_t r0, int64_t r1, const int64_t* rowptr,
               const int64_t* colind, const double* val, int64_t base_ptr, int64_t base_idx) {
  free_run(ctx);
  free_matrix(ctx);
  const int64_t m = r1 - r0;
  const int64_t nnz = rowptr[m] - rowptr[0];
  std::vector<int64_t> rp(m + 1);
  for (int64_t i = 0; i <= m; ++i) rp[i] = rowptr[i] - rowptr[0];
  std::vector<int32_t> ci(nnz);
  const int64_t e0 = rowptr[0] - base_ptr;
  for (int64_t e = 0; e < nnz; ++e) {
    const int64_t c = colind[e0 + e] - base_idx;
    if (c < 0 || c >= n) return fail(ctx, RBL_ERR_INVALID, "column index out of range");
    if (c > INT32_MAX) return fail(ctx, RBL_ERR_INVALID, "n exceeds int32 column ids");
    ci[e] = (int32_t)c;
  }
  // rows must be column-sorted (SparseArrays guarantees it; the window kernel relies on it)
  for (int64_t i = 0; i < m; ++i)
    for (int64_t e = rp[i] + 1; e < rp[i + 1]; ++e)
      if (ci[e] < ci[e - 1]) return fail(ctx, RBL_ERR_INVALID, "row indices not sorted");
  ctx->n = n;
  ctx->r0 = r0;
  ctx->r1 = r1;
  ctx->nloc = m;
  ctx->nnz = nnz;
  HIPC(hipMalloc(&ctx->d_rowptr, (m + 1) * sizeof(int64_t)));
  HIPC(hipMalloc(&ctx->d_col, (nnz + kCsrPad) * sizeof(int32_t)));
  HIPC(hipMalloc(&ctx->d_val, (nnz + kCsrPad) * sizeof(double)));
  HIPC(hipMemset(ctx->d_col + nnz, 0, kCsrPad * sizeof(int32_t)));
  HIPC(hipMemset(ctx->d_val + nnz, 0, kCsrPad * sizeof(double)));
  HIPC(hipMemcpy(ctx->d_rowptr, rp.data(), (m + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  if (nnz) {
    HIPC(hipMemcpy(ctx->d_col, ci.data(), nnz * sizeof(int32_t), hipMemcpyHostToDevice));
    HIPC(hipMemcpy(ctx->d_val, val + e0, nnz * sizeof(double), hipMemcpyHostToDevice));
  }
  // halo needs: column footprint per owning rank
  const int P = ctx->nranks;
  ctx->need_lo.assign(P, 0);
  ctx->need_hi.assign(P, 0);
  if (P > 1) {
    std::vector<int64_t> lo(P), hi(P);
    for (int q = 0; q < P; ++q) { lo[q] = INT64_MAX; hi[q] = -1; }
    for (int64_t e = 0; e < nnz; ++e) {
      const int64_t c = ci[e];
      const int q = (int)(std::upper_bound(ctx->bounds.begin(), ctx->bounds.end(), c) -
                          ctx->bounds.begin()) - 1;
      lo[q] = std::min(lo[q], c);
      hi[q] = std::max(hi[q], c + 1);
    }
    for (int q = 0; q < P; ++q) {
      ctx->need_lo[q] = hi[q] < 0 ? 0 : lo[q];
      ctx->need_hi[q] = hi[q] < 0 ? 0 : hi[q];
    }
  }
  CHK(prepare_window(ctx, rp));
  return setup_halo(ctx);
}

// The halo of an unbanded local CSR (R-MAT, circuit): for every other rank q, the contiguous
// range of q's rows the local columns reference (col_footprint on the device).
int halo_from_footprint(rbl_ctx* ctx) {
  const int P = ctx->nranks;
  const int64_t nnz = ctx->nnz;
  ctx->need_lo.assign(P, 0);
  ctx->need_hi.assign(P, 0);
  if (P > 1 && nnz > 0) {
    int64_t* d_b = nullptr;
    unsigned long long* d_lh = nullptr;
    HIPC(hipMalloc(&d_b, (P + 1) * sizeof(int64_t)));
    HIPC(hipMalloc(&d_lh, 2 * P * sizeof(unsigned long long)));
    std::vector<unsigned long long> lh(2 * P);
    for (int q = 0; q < P; ++q) { lh[q] = ~0ull; lh[P + q] = 0ull; }
    HIPC(hipMemcpy(d_b, ctx->bounds.data(), (P + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
    HIPC(hipMemcpy(d_lh, lh.data(), 2 * P * sizeof(unsigned long long), hipMemcpyHostToDevice));
    col_footprint(ctx->d_col, nnz, d_b, P, d_lh, d_lh + P, ctx->stream);
    HIPC(hipGetLastError());
    HIPC(hipMemcpyAsync(lh.data(), d_lh, 2 * P * sizeof(unsigned long long), hipMemcpyDeviceToHost, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    hipFree(d_b);
    hipFree(d_lh);
    for (int q = 0; q < P; ++q) {
      if (q == ctx->rank || lh[P + q] == 0ull) continue;
      ctx->need_lo[q] = (int64_t)lh[q];
      ctx->need_hi[q] = (int64_t)lh[P + q];
    }
  }
  return RBL_OK;
}

}  // namespace

// =========================================================================================
extern "C" {

int rbl_abi_version(void) { return RBL_ABI_VERSION; }
int rbl_build_flags(void) {
#ifdef RBL_VARIANTS
  return RBL_BUILD_VARIANTS;
#else
  return 0;
#endif
}

int rbl_create(rbl_ctx** out, int device) {
  if (!out) return RBL_ERR_INVALID;
  rbl_ctx* ctx = new rbl_ctx();
  ctx->device = device;
  *out = ctx;
  HIPC(hipSetDevice(device));
  HIPC(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
  ctx->bounds = {0, 0};
  return RBL_OK;
}

int rbl_get_unique_id(uint8_t unique_id[128]) {
  if (!unique_id) return RBL_ERR_INVALID;
  return rccl_unique_id(unique_id) == 0 ? RBL_OK : RBL_ERR_RCCL;
}

int rbl_comm_selftest(int device, char* msg, int msg_len) {
  // one-rank RCCL communicator through the production transport (RcclComm): the three
  // collective shapes on real device buffers, checked on the host
  std::string err;
  auto say = [&](const std::string& m) {
    if (msg && msg_len > 0) snprintf(msg, (size_t)msg_len, "%s", m.c_str());
  };
  if (hipSetDevice(device) != hipSuccess) { say("hipSetDevice failed"); return RBL_ERR_HIP; }
  uint8_t id[128];
  if (rccl_unique_id(id) != 0) { say("ncclGetUniqueId failed"); return RBL_ERR_RCCL; }
  Comm* c = make_rccl_comm(1, 0, id, &err);
  if (!c) { say("ncclCommInitRank: " + err); return RBL_ERR_RCCL; }
  hipStream_t st = nullptr;
  double* d = nullptr;
  int rc = RBL_OK;
  const size_t n = 4096;
  std::vector<double> h(n), back(n);
  for (size_t k = 0; k < n; ++k) h[k] = 0.5 * (double)k - 7.0;
  if (hipStreamCreate(&st) != hipSuccess || hipMalloc(&d, 2 * n * sizeof(double)) != hipSuccess ||
      hipMemcpy(d, h.data(), n * sizeof(double), hipMemcpyHostToDevice) != hipSuccess) {
    say("HIP setup failed");
    rc = RBL_ERR_HIP;
  }
  if (rc == RBL_OK && c->allreduce_sum(d, n, st, &err) != 0) { say("allreduce: " + err); rc = RBL_ERR_RCCL; }
  if (rc == RBL_OK) {
    hipMemcpyAsync(back.data(), d, n * sizeof(double), hipMemcpyDeviceToHost, st);
    hipStreamSynchronize(st);
    if (back != h) { say("allreduce over one rank changed the data"); rc = RBL_ERR_RCCL; }
  }
  int64_t mine[3] = {11, -2, 1LL << 40}, all[3] = {0, 0, 0};
  if (rc == RBL_OK && c->allgather_host(mine, all, 3, st, &err) != 0) { say("allgather: " + err); rc = RBL_ERR_RCCL; }
  if (rc == RBL_OK && (all[0] != mine[0] || all[1] != mine[1] || all[2] != mine[2])) {
    say("allgather returned other values");
    rc = RBL_ERR_RCCL;
  }
  std::vector<Comm::Xfer> x(1);  // no peers: an empty grouped exchange
  if (rc == RBL_OK && c->exchange(x, st, &err) != 0) { say("exchange: " + err); rc = RBL_ERR_RCCL; }
  if (rc == RBL_OK && hipStreamSynchronize(st) != hipSuccess) { say("stream sync failed"); rc = RBL_ERR_HIP; }
  if (rc == RBL_OK) say(std::string("ok: ") + c->name());
  delete c;
  if (d) (void)hipFree(d);
  if (st) (void)hipStreamDestroy(st);
  return rc;
}

int rbl_create_dist(rbl_ctx** out, int device, int nranks, int rank, const uint8_t unique_id[128]) {
  if (!out || nranks < 1 || rank < 0 || rank >= nranks) return RBL_ERR_INVALID;
  int s = rbl_create(out, device);
  if (s != RBL_OK) return s;
  rbl_ctx* ctx = *out;
  ctx->nranks = nranks;
  ctx->rank = rank;
  if (nranks > 1) {
    if (!unique_id) return fail(ctx, RBL_ERR_INVALID, "rbl_create_dist: null unique_id");
    ctx->comm = make_rccl_comm(nranks, rank, unique_id, &ctx->err);
    if (!ctx->comm) return RBL_ERR_RCCL;
  }
  return RBL_OK;
}

int rbl_local_group_create(rbl_group** group, int nranks) {
  if (!group || nranks < 1) return RBL_ERR_INVALID;
  *group = reinterpret_cast<rbl_group*>(local_group_create(nranks));
  return RBL_OK;
}

int rbl_local_group_free(rbl_group* group) {
  local_group_release(reinterpret_cast<LocalGroup*>(group));
  return RBL_OK;
}

int rbl_create_local(rbl_ctx** out, int device, rbl_group* group, int rank) {
  if (!out || !group) return RBL_ERR_INVALID;
  int s = rbl_create(out, device);
  if (s != RBL_OK) return s;
  rbl_ctx* ctx = *out;
  ctx->comm = make_local_comm(reinterpret_cast<LocalGroup*>(group), rank, &ctx->err);
  if (!ctx->comm) return RBL_ERR_INVALID;
  ctx->nranks = ctx->comm->nranks;
  ctx->rank = rank;
  return RBL_OK;
}

int rbl_create_shm(rbl_ctx** out, int device, int nranks, int rank, const char* path) {
  if (!out || nranks < 1 || rank < 0 || rank >= nranks || !path) return RBL_ERR_INVALID;
  int s = rbl_create(out, device);
  if (s != RBL_OK) return s;
  rbl_ctx* ctx = *out;
  ctx->nranks = nranks;
  ctx->rank = rank;
  if (nranks > 1) {
    ctx->comm = make_shm_comm(nranks, rank, path, &ctx->err);
    if (!ctx->comm) return RBL_ERR_RCCL;
  }
  return RBL_OK;
}

int rbl_free(rbl_ctx* ctx) {
  if (!ctx) return RBL_OK;
  hipSetDevice(ctx->device);
  if (ctx->stream) hipStreamSynchronize(ctx->stream);
  if (ctx->hstream) hipStreamSynchronize(ctx->hstream);
  free_run(ctx);
  free_matrix(ctx);
  for (auto e : ctx->ev_pool) hipEventDestroy(e);
  for (auto e : ctx->step_ev)
    if (e) hipEventDestroy(e);
  delete ctx->comm;
  if (ctx->stream) hipStreamDestroy(ctx->stream);
  if (ctx->cstream) hipStreamDestroy(ctx->cstream);
  if (ctx->hstream) hipStreamDestroy(ctx->hstream);
  if (ctx->rstream) hipStreamDestroy(ctx->rstream);
  for (hipEvent_t e : ctx->ev_ritz)
    if (e) hipEventDestroy(e);
  if (ctx->ev_push_ready) hipEventDestroy(ctx->ev_push_ready);
  if (ctx->ev_push_done) hipEventDestroy(ctx->ev_push_done);
  for (hipEvent_t e : {ctx->ev_fin, ctx->ev_d2h[0], ctx->ev_d2h[1], ctx->ev_d2h_slot[0],
                       ctx->ev_d2h_slot[1], ctx->ev_qready, ctx->ev_halo})
    if (e) hipEventDestroy(e);
  for (void* h : ctx->h_d2h)
    if (h) hipHostFree(h);
  delete ctx;
  return RBL_OK;
}

const char* rbl_last_error(const rbl_ctx* ctx) { return ctx ? ctx->err.c_str() : "null context"; }

int rbl_device_memory(rbl_ctx* ctx, int64_t* free_bytes, int64_t* total_bytes) {
  if (!ctx || !free_bytes || !total_bytes) return RBL_ERR_INVALID;
  HIPC(hipSetDevice(ctx->device));
  size_t fr = 0, tot = 0;
  HIPC(hipMemGetInfo(&fr, &tot));
  *free_bytes = (int64_t)fr;
  *total_bytes = (int64_t)tot;
  return RBL_OK;
}

int rbl_comm_info(rbl_ctx* ctx, int* nranks, int* rank, char* transport, int transport_len) {
  if (!ctx || !nranks || !rank) return RBL_ERR_INVALID;
  int cnt = 1;
  const char* name = "none";
  if (ctx->comm) {
    hipSetDevice(ctx->device);
    const int s = ctx->comm->count(&cnt, &ctx->err);
    if (s < 0) return s;
    name = ctx->comm->name();
  }
  *nranks = cnt;
  *rank = ctx->rank;
  if (transport && transport_len > 0) snprintf(transport, (size_t)transport_len, "%s", name);
  return RBL_OK;
}

int rbl_rccl_version(int* version, char* path, int path_len) {
  if (!version) return RBL_ERR_INVALID;
  std::string p, err;
  const int s = rbl::rccl_library(version, &p, &err);
  if (path && path_len > 0) snprintf(path, (size_t)path_len, "%s", s ? err.c_str() : p.c_str());
  return s ? RBL_ERR_RCCL : RBL_OK;
}

int rbl_set_option(rbl_ctx* ctx, int option, int64_t value) {
  if (!ctx) return RBL_ERR_INVALID;
  switch (option) {
    case RBL_OPT_TIMERS:
      if (value < 0 || value > 2) return fail(ctx, RBL_ERR_INVALID, "RBL_OPT_TIMERS: 0, 1 or 2");
      ctx->timers = (int)value;
      return RBL_OK;
    case RBL_OPT_REORTH_ORDER:
      if (value < 0 || value > 1) return fail(ctx, RBL_ERR_INVALID, "reorth order must be 0|1");
      ctx->reorth_order = (int)value;
      return RBL_OK;
    case RBL_OPT_DEVICE_BLOCKS:
      if (value < -1 || value == 1 || value == 2 || value > INT32_MAX)
        return fail(ctx, RBL_ERR_INVALID, "device blocks: 0 (all), -1 (auto) or >= 3");
      ctx->dev_blocks_opt = (int)value;
      return RBL_OK;
    case RBL_OPT_SPMM_KERNEL:
      // option values are the kernel ids rbl_spmm_kernel_for reports (4, the dense panel GEMM,
      // follows from rbl_set_matrix_dense and is not selectable); internally the band tiles
      // are variant 4 and the segmented gather variant 5 (spmm.hip)
      if (value < 0 || value > 7 || value == 4)
        return fail(ctx, RBL_ERR_INVALID, "spmm kernel must be 0 (auto) or a kernel id 1, 2, 3, 5, 6, 7");
      ctx->spmm_variant = value == 5 ? 4 : value == 6 ? 5 : (int)value;
      return RBL_OK;
    case RBL_OPT_SPLIT_HALO: ctx->split_halo = value != 0; return RBL_OK;
    case RBL_OPT_HALO_OVERLAP: ctx->halo_overlap = value != 0; return RBL_OK;
    case RBL_OPT_HALO_PUSH:
      if (value < 0 || value > 2) return fail(ctx, RBL_ERR_INVALID, "RBL_OPT_HALO_PUSH must be 0|1|2");
      ctx->halo_push_opt = (int)value;
      return RBL_OK;
    case RBL_OPT_KEEP_CSR: ctx->keep_csr = value != 0; return RBL_OK;
    case RBL_OPT_RELABEL:
      if (value < 0 || value > 1) return fail(ctx, RBL_ERR_INVALID, "RBL_OPT_RELABEL must be 0|1");
      ctx->relabel_opt = (int)value;
      return RBL_OK;
    case RBL_OPT_FUSE:
      if (value < 0 || value > 7) return fail(ctx, RBL_ERR_INVALID, "RBL_OPT_FUSE is a 3-bit mask");
      ctx->fuse = (int)value;
      return RBL_OK;
    default: return fail(ctx, RBL_ERR_INVALID, "unknown option");
  }
}

int rbl_set_matrix_csc(rbl_ctx* ctx, int64_t n, int64_t nnz, const int64_t* colptr,
                       const int64_t* rowval, const double* nzval, int index_base) {
  if (!ctx || n < 1 || nnz < 0 || !colptr || (nnz && (!rowval || !nzval)) ||
      (index_base != 0 && index_base != 1))
    return fail(ctx, RBL_ERR_INVALID, "rbl_set_matrix_csc: bad arguments");
  if (colptr[n] - colptr[0] != nnz) return fail(ctx, RBL_ERR_INVALID, "colptr[n] != nnz");
  HIPC(hipSetDevice(ctx->device));
  // symmetric: column slice [r0,r1) of CSC == row slice of CSR
  std::vector<int64_t> rp(n + 1);
  for (int64_t i = 0; i <= n; ++i) rp[i] = colptr[i] - colptr[0];
  ctx->bounds.assign(ctx->nranks + 1, 0);
  rbl_plan_row_partition(n, rp.data(), ctx->nranks, ctx->bounds.data());
  const int64_t r0 = ctx->bounds[ctx->rank], r1 = ctx->bounds[ctx->rank + 1];
  return upload_csr(ctx, n, r0, r1, colptr + r0, rowval, nzval, index_base, index_base);
}

int rbl_set_matrix_csr_rows(rbl_ctx* ctx, int64_t n, int64_t row_begin, int64_t row_end,
                            const int64_t* rowptr, const int64_t* colind, const double* val,
                            int index_base) {
  if (!ctx || n < 1 || row_begin < 0 || row_end < row_begin || row_end > n || !rowptr ||
      (index_base != 0 && index_base != 1))
    return fail(ctx, RBL_ERR_INVALID, "rbl_set_matrix_csr_rows: bad arguments");
  HIPC(hipSetDevice(ctx->device));
  // the partition is the callers' (every rank's [row_begin,row_end) must tile [0,n))
  if (ctx->nranks > 1) {
    int64_t mine[2] = {row_begin, row_end};
    std::vector<int64_t> all(2 * ctx->nranks);
    COMMC(ctx->comm->allgather_host(mine, all.data(), 2, ctx->stream, &ctx->err));
    ctx->bounds.assign(ctx->nranks + 1, 0);
    for (int p = 0; p < ctx->nranks; ++p) {
      if (all[2 * p] != (p == 0 ? 0 : all[2 * p - 1]))
        return fail(ctx, RBL_ERR_INVALID, "row slices must tile [0,n) in rank order");
      ctx->bounds[p + 1] = all[2 * p + 1];
    }
    if (ctx->bounds[ctx->nranks] != n) return fail(ctx, RBL_ERR_INVALID, "row slices != n");
  } else {
    if (row_begin != 0 || row_end != n)
      return fail(ctx, RBL_ERR_INVALID, "single rank must own all rows");
    ctx->bounds = {0, n};
  }
  return upload_csr(ctx, n, row_begin, row_end, rowptr, colind, val, index_base, index_base);
}

int rbl_set_matrix_dense(rbl_ctx* ctx, int64_t n, int64_t row_begin, int64_t row_end,
                         const double* A, int64_t lda) {
  if (!ctx || n < 1 || row_begin < 0 || row_end < row_begin || row_end > n || !A ||
      lda < row_end - row_begin || lda < 1)
    return fail(ctx, RBL_ERR_INVALID, "rbl_set_matrix_dense: bad arguments");
  HIPC(hipSetDevice(ctx->device));
  free_run(ctx);
  free_matrix(ctx);
  ctx->bounds.assign(ctx->nranks + 1, 0);
  if (ctx->nranks > 1) {  // the row slices must tile [0, n) in rank order
    int64_t mine[2] = {row_begin, row_end};
    std::vector<int64_t> all(2 * ctx->nranks);
    COMMC(ctx->comm->allgather_host(mine, all.data(), 2, ctx->stream, &ctx->err));
    for (int p = 0; p < ctx->nranks; ++p) {
      if (all[2 * p] != (p == 0 ? 0 : all[2 * p - 1]))
        return fail(ctx, RBL_ERR_INVALID, "row slices must tile [0,n) in rank order");
      ctx->bounds[p + 1] = all[2 * p + 1];
    }
    if (ctx->bounds[ctx->nranks] != n) return fail(ctx, RBL_ERR_INVALID, "row slices != n");
  } else {
    if (row_begin != 0 || row_end != n) return fail(ctx, RBL_ERR_INVALID, "one rank holds all rows");
    ctx->bounds[1] = n;
  }
  const int64_t m = row_end - row_begin;
  ctx->n = n;
  ctx->r0 = row_begin;
  ctx->r1 = row_end;
  ctx->nloc = m;
  ctx->nnz = m * n;
  ctx->dense = true;
  ctx->dense_panels = (n + 31) / 32;
  const int64_t P = ctx->dense_panels;
  const int64_t ml = std::max<int64_t>(m, 1);
  HIPC(hipMalloc(&ctx->d_dense, (size_t)P * ml * 32 * sizeof(double)));
  HIPC(hipMalloc(&ctx->d_qfull, (size_t)P * 32 * 64 * sizeof(double)));
  HIPC(hipMemsetAsync(ctx->d_qfull, 0, (size_t)P * 32 * 64 * sizeof(double), ctx->stream));
  ctx->qfull_cols = 64;
  // column-major slice -> row-major 32-column panels, one panel at a time through a scratch
  double* d_tmp = nullptr;
  HIPC(hipMalloc(&d_tmp, (size_t)ml * 32 * sizeof(double)));
  for (int64_t p = 0; p < P && m > 0; ++p) {
    const int64_t c0 = 32 * p, nc = std::min<int64_t>(32, n - c0);
    if (nc < 32) HIPC(hipMemsetAsync(d_tmp, 0, (size_t)m * 32 * sizeof(double), ctx->stream));
    HIPC(hipMemcpy2DAsync(d_tmp, m * sizeof(double), A + c0 * lda, lda * sizeof(double),
                          m * sizeof(double), nc, hipMemcpyHostToDevice, ctx->stream));
    colmajor_to_rowmajor(d_tmp, m, 32, ctx->d_dense + p * m * 32, ctx->stream);
  }
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(ctx->stream));
  hipFree(d_tmp);
  // every rank needs all n rows of Q
  const int Pr = ctx->nranks;
  ctx->need_lo.assign(Pr, 0);
  ctx->need_hi.assign(Pr, 0);
  for (int q = 0; q < Pr; ++q) {
    ctx->need_lo[q] = ctx->bounds[q];
    ctx->need_hi[q] = ctx->bounds[q + 1];
  }
  return setup_halo(ctx);
}

int rbl_gen_matrix_hashwindow(rbl_ctx* ctx, int64_t n, int64_t halfwidth, double density,
                              uint64_t seed, int nplant, const double* plant) {
  if (!ctx || n < 1 || halfwidth < 0 || nplant < 0 || (nplant > 0 && !plant) || n > INT32_MAX)
    return fail(ctx, RBL_ERR_INVALID, "rbl_gen_matrix_hashwindow: bad arguments");
  HIPC(hipSetDevice(ctx->device));
  free_run(ctx);
  free_matrix(ctx);
  const int P = ctx->nranks;
  ctx->bounds.assign(P + 1, 0);
  for (int p = 0; p <= P; ++p) ctx->bounds[p] = n * p / P;  // uniform rows: ~uniform nnz
  const int64_t r0 = ctx->bounds[ctx->rank], r1 = ctx->bounds[ctx->rank + 1], m = r1 - r0;
  ctx->n = n;
  ctx->r0 = r0;
  ctx->r1 = r1;
  ctx->nloc = m;
  int32_t* d_cnt = nullptr;
  HIPC(hipMalloc(&d_cnt, std::max<int64_t>(m, 1) * sizeof(int32_t)));
  hw_count(n, halfwidth, density, seed, r0, r1, d_cnt, ctx->stream);
  std::vector<int32_t> cnt(m);
  HIPC(hipMemcpyAsync(cnt.data(), d_cnt, m * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  hipFree(d_cnt);
  std::vector<int64_t> rp(m + 1, 0);
  for (int64_t i = 0; i < m; ++i) rp[i + 1] = rp[i] + cnt[i];
  ctx->nnz = rp[m];
  HIPC(hipMalloc(&ctx->d_rowptr, (m + 1) * sizeof(int64_t)));
  HIPC(hipMalloc(&ctx->d_col, (ctx->nnz + kCsrPad) * sizeof(int32_t)));
  HIPC(hipMalloc(&ctx->d_val, (ctx->nnz + kCsrPad) * sizeof(double)));
  HIPC(hipMemset(ctx->d_col + ctx->nnz, 0, kCsrPad * sizeof(int32_t)));
  HIPC(hipMemset(ctx->d_val + ctx->nnz, 0, kCsrPad * sizeof(double)));
  HIPC(hipMemcpy(ctx->d_rowptr, rp.data(), (m + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  double* d_plant = nullptr;
  if (nplant > 0) {
    HIPC(hipMalloc(&d_plant, nplant * sizeof(double)));
    HIPC(hipMemcpy(d_plant, plant, nplant * sizeof(double), hipMemcpyHostToDevice));
  }
  hw_fill(n, halfwidth, density, seed, r0, r1, ctx->d_rowptr, nplant, d_plant, ctx->d_col,
          ctx->d_val, ctx->stream);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(ctx->stream));
  hipFree(d_plant);
  ctx->need_lo.assign(P, 0);
  ctx->need_hi.assign(P, 0);
  for (int q = 0; q < P; ++q) {  // analytic footprint of the window
    const int64_t lo = std::max(ctx->bounds[q], std::max<int64_t>(0, r0 - halfwidth));
    const int64_t hi = std::min(ctx->bounds[q + 1], std::min<int64_t>(n, r1 + halfwidth));
    if (hi > lo && q != ctx->rank) {
      ctx->need_lo[q] = lo;
      ctx->need_hi[q] = hi;
    }
  }
  CHK(prepare_window(ctx, rp));
  return setup_halo(ctx);
}

int rbl_gen_matrix_circuit(rbl_ctx* ctx, int64_t n, int64_t width, double p_edge, uint64_t seed,
                           int nplant, const double* plant) {
  if (!ctx || n < 1 || width < 1 || nplant < 0 || (nplant > 0 && !plant) || n > INT32_MAX ||
      !(p_edge >= 0.0 && p_edge <= 1.0))
    return fail(ctx, RBL_ERR_INVALID, "rbl_gen_matrix_circuit: bad arguments");
  HIPC(hipSetDevice(ctx->device));
  free_run(ctx);
  free_matrix(ctx);
  const int P = ctx->nranks;
  ctx->bounds.assign(P + 1, 0);
  for (int q = 0; q <= P; ++q) ctx->bounds[q] = n * q / P;  // <= 5 nonzeros per row: uniform
  const int64_t r0 = ctx->bounds[ctx->rank], r1 = ctx->bounds[ctx->rank + 1], m = r1 - r0;
  ctx->n = n;
  ctx->r0 = r0;
  ctx->r1 = r1;
  ctx->nloc = m;
  int32_t* d_cnt = nullptr;
  HIPC(hipMalloc(&d_cnt, std::max<int64_t>(m, 1) * sizeof(int32_t)));
  circ_count(n, width, p_edge, seed, r0, r1, d_cnt, ctx->stream);
  HIPC(hipGetLastError());
  std::vector<int32_t> cnt(m);
  HIPC(hipMemcpyAsync(cnt.data(), d_cnt, m * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  hipFree(d_cnt);
  std::vector<int64_t> rp(m + 1, 0);
  for (int64_t i = 0; i < m; ++i) rp[i + 1] = rp[i] + cnt[i];
  ctx->nnz = rp[m];
  HIPC(hipMalloc(&ctx->d_rowptr, (m + 1) * sizeof(int64_t)));
  HIPC(hipMalloc(&ctx->d_col, (ctx->nnz + kCsrPad) * sizeof(int32_t)));
  HIPC(hipMalloc(&ctx->d_val, (ctx->nnz + kCsrPad) * sizeof(double)));
  HIPC(hipMemset(ctx->d_col + ctx->nnz, 0, kCsrPad * sizeof(int32_t)));
  HIPC(hipMemset(ctx->d_val + ctx->nnz, 0, kCsrPad * sizeof(double)));
  HIPC(hipMemcpy(ctx->d_rowptr, rp.data(), (m + 1) * sizeof(int64_t), hipMemcpyHostToDevice));
  double* d_plant = nullptr;
  if (nplant > 0) {
    HIPC(hipMalloc(&d_plant, nplant * sizeof(double)));
    HIPC(hipMemcpy(d_plant, plant, nplant * sizeof(double), hipMemcpyHostToDevice));
  }
  circ_fill(n, width, p_edge, seed, r0, r1, ctx->d_rowptr, nplant, d_plant, ctx->d_col,
            ctx->d_val, ctx->stream);
  HIPC(hipGetLastError());
  HIPC(hipStreamSynchronize(ctx->stream));
  hipFree(d_plant);
  CHK(halo_from_footprint(ctx));
  CHK(prepare_window(ctx, rp));
  return setup_halo(ctx);
}

int rbl_gen_matrix_rmat(rbl_ctx* ctx, int64_t n, int scale, int64_t edges, double a, double b,
                        double c, uint64_t seed, int nplant, const double* plant) {
  if (!ctx || n < 1 || scale < 1 || scale > 31 || ((int64_t)1 << scale) < n || edges < 0 ||
      a < 0 || b < 0 || c < 0 || a + b + c > 1.0 || nplant < 0 || (nplant > 0 && !plant) ||
      n > INT32_MAX)
    return fail(ctx, RBL_ERR_INVALID, "rbl_gen_matrix_rmat: bad arguments");
  if (ctx->nranks > 16) return fail(ctx, RBL_ERR_INVALID, "rbl_gen_matrix_rmat: at most 16 ranks");
  HIPC(hipSetDevice(ctx->device));
  free_run(ctx);
  free_matrix(ctx);
  RmatParams p;
  p.n = n;
  p.scale = scale;
  p.edges = edges;
  p.a = a;
  p.b = b;
  p.c = c;
  p.seed = seed;
  p.relabel = ctx->relabel_opt != 0;
  if (p.relabel) p.perm = make_scatter(n, seed ^ kRelabelK);
  // degrees of every row (all ranks draw every edge): they size the key buffer and balance
  // the row split by nonzeros (R-MAT's low ids are its hubs)
  int32_t* d_deg = nullptr;
  HIPC(hipMalloc(&d_deg, n * sizeof(int32_t)));
  HIPC(hipMemsetAsync(d_deg, 0, n * sizeof(int32_t), ctx->stream));
  rmat_degree(p, d_deg, ctx->stream);
  HIPC(hipGetLastError());
  std::vector<int32_t> deg(n);
  HIPC(hipMemcpyAsync(deg.data(), d_deg, n * sizeof(int32_t), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  hipFree(d_deg);
  const int P = ctx->nranks;
  std::vector<int64_t> pre(n + 1, 0);  // nonzeros (with duplicates) + diagonal, prefix
  for (int64_t r = 0; r < n; ++r) pre[r + 1] = pre[r] + deg[r] + 1;
  ctx->bounds.assign(P + 1, 0);
  ctx->bounds[P] = n;
  for (int q = 1; q < P; ++q) {
    const int64_t target = pre[n] * q / P;
    ctx->bounds[q] = std::lower_bound(pre.begin(), pre.end(), target) - pre.begin();
    ctx->bounds[q] = std::max(ctx->bounds[q], ctx->bounds[q - 1]);
  }
  const int64_t r0 = ctx->bounds[ctx->rank], r1 = ctx->bounds[ctx->rank + 1], m = r1 - r0;
  ctx->n = n;
  ctx->r0 = r0;
  ctx->r1 = r1;
  ctx->nloc = m;
  int64_t own = 0;
  for (int64_t r = r0; r < r1; ++r) own += deg[r];
  double* d_plant = nullptr;
  if (nplant > 0) {
    HIPC(hipMalloc(&d_plant, nplant * sizeof(double)));
    HIPC(hipMemcpy(d_plant, plant, nplant * sizeof(double), hipMemcpyHostToDevice));
  }
  HIPC(hipMalloc(&ctx->d_rowptr, (m + 1) * sizeof(int64_t)));
  int64_t nnz = 0;
  const int st = rmat_local_csr(p, r0, r1, own, nplant, d_plant, ctx->d_rowptr, &ctx->d_col,
                                &ctx->d_val, &nnz, ctx->stream);
  hipFree(d_plant);
  ctx->relabeled = p.relabel;
  ctx->relabel_perm = p.perm;
  if (st == -1) return fail(ctx, RBL_ERR_INVALID, "rbl_gen_matrix_rmat: > 2^31 keys on one rank");
  if (st < 0) return fail(ctx, st == -3 ? RBL_ERR_OOM : RBL_ERR_HIP, "rbl_gen_matrix_rmat: device generation failed");
  ctx->nnz = nnz;
  std::vector<int64_t> rp(m + 1);
  HIPC(hipMemcpy(rp.data(), ctx->d_rowptr, (m + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
  CHK(halo_from_footprint(ctx));
  CHK(prepare_window(ctx, rp));
  return setup_halo(ctx);
}

int rbl_matrix_info(rbl_ctx* ctx, int64_t* n, int64_t* row_begin, int64_t* row_end,
                    int64_t* nnz_local) {
  if (!ctx) return RBL_ERR_INVALID;
  if (n) *n = ctx->n;
  if (row_begin) *row_begin = ctx->r0;
  if (row_end) *row_end = ctx->r1;
  if (nnz_local) *nnz_local = ctx->nnz;
  return RBL_OK;
}

int rbl_row_ids(rbl_ctx* ctx, int64_t* ids) {
  if (!ctx || !ids) return RBL_ERR_INVALID;
  if (!has_matrix(ctx)) return fail(ctx, RBL_ERR_STATE, "rbl_row_ids: no matrix");
  for (int64_t i = 0; i < ctx->nloc; ++i)
    ids[i] = ctx->relabeled ? scatter_inv(ctx->relabel_perm, ctx->r0 + i) : ctx->r0 + i;
  return RBL_OK;
}

int rbl_get_matrix_csr(rbl_ctx* ctx, int64_t* rowptr, int32_t* colind, double* val) {
  if (ctx && ctx->csr_dropped)
    return fail(ctx, RBL_ERR_STATE, "rbl_get_matrix_csr: the CSR was released (RBL_OPT_KEEP_CSR = 0)");
  if (!ctx || !ctx->d_rowptr)
    return fail(ctx, RBL_ERR_STATE, ctx && ctx->dense ? "dense matrix: no CSR" : "no matrix");
  HIPC(hipSetDevice(ctx->device));
  if (rowptr)
    HIPC(hipMemcpy(rowptr, ctx->d_rowptr, (ctx->nloc + 1) * sizeof(int64_t), hipMemcpyDeviceToHost));
  if (colind && ctx->nnz)
    HIPC(hipMemcpy(colind, ctx->d_col, ctx->nnz * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (val && ctx->nnz)
    HIPC(hipMemcpy(val, ctx->d_val, ctx->nnz * sizeof(double), hipMemcpyDeviceToHost));
  return RBL_OK;
}

int rbl_spmm_kernel_for(rbl_ctx* ctx, int b) {
  if (!ctx || !has_matrix(ctx)) return RBL_ERR_INVALID;
  if (ctx->dense) return 4;
  if (ctx->spmm_variant == 1) return 1;
  const int v = ctx->spmm_variant;
  const bool band = ctx->ntiles > 0 && ((b == 16 && ctx->band_ok16) || (b == 32 && ctx->band_ok32));
  const bool win = ctx->ntiles > 0 && ((b == 16 && ctx->window_ok16) || (b == 32 && ctx->window_ok32));
  const bool panel = b == 32 && ctx->panel_nblk > 0 && !ctx->csr_dropped && !ctx->ghost;
  if ((v == 0 || v == 4) && (b == 32 || b == 16) && (ctx->bt_ng == 5 || ctx->bt_ng == 9)) return 5;
  if ((v == 0 || v == 3 || v == 4) && band) return 3;
  if (((v == 0 && ctx->panel_auto) || v == 7) && panel) return 7;
  if ((v == 0 || v == 2 || v == 3) && win) return 2;
  if ((v == 0 || v == 5) && ctx->seg_ntasks > 0 && (b == 16 || b == 32)) return 6;
  return 1;
}

int rbl_matrix_format(rbl_ctx* ctx) {
  if (!ctx || !has_matrix(ctx)) return RBL_ERR_INVALID;
  if (ctx->dense) return 4;
  if (ctx->d_bth) return 3;
  if (ctx->d_btp_hdr) return 2;
  if (ctx->d_bt) return 1;
  return 0;
}

int rbl_apply(rbl_ctx* ctx, int b, const double* X, double* Y) {
  if (!ctx || b < 1 || b > RBL_MAX_BLOCK || !X || !Y) return fail(ctx, RBL_ERR_INVALID, "rbl_apply: bad arguments");
  if (!has_matrix(ctx)) return fail(ctx, RBL_ERR_STATE, "rbl_apply: no matrix");
  if (ctx->b != 0 && ctx->b != b && ctx->nranks > 1)
    return fail(ctx, RBL_ERR_STATE, "rbl_apply: b differs from the running Krylov block size");
  HIPC(hipSetDevice(ctx->device));
  const int64_t nl = std::max<int64_t>(ctx->nloc, 1);
  DevBuf x, xr, y, ext;
  HIPC(hipMalloc(&x.p, nl * b * sizeof(double)));
  HIPC(hipMalloc(&xr.p, nl * b * sizeof(double)));
  HIPC(hipMalloc(&y.p, (nl + kRowPad) * b * sizeof(double)));
  HIPC(hipMemcpyAsync(x.p, X, ctx->nloc * b * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
  colmajor_to_rowmajor(x.d(), ctx->nloc, b, xr.d(), ctx->stream);
  const double* Qin = xr.d();
  int64_t off = 0;
  DevBuf sendbuf;
  if (ctx->nranks > 1) {  // halo exchange through a private extended buffer
    const int64_t ext_rows = qext_rows(ctx, b);
    HIPC(hipMalloc(&ext.p, ext_rows * b * sizeof(double)));
    // rows between the received ranges stay finite (band-tile kernel multiplies them by 0)
    HIPC(hipMemsetAsync(ext.p, 0, ext_rows * b * sizeof(double), ctx->stream));
    if (use_ghost(ctx, b))
      HIPC(hipMalloc(&sendbuf.p, std::max<int64_t>(ctx->n_send, 1) * b * sizeof(double)));
    double* keep_ext = ctx->d_qext;
    const size_t keep_cap = ctx->qext_cap;
    double* keep_send = ctx->d_sendbuf;
    const int keep_b = ctx->b;
    ctx->d_qext = ext.d();
    ctx->qext_cap = (size_t)ext_rows * b;
    ctx->d_sendbuf = sendbuf.d();
    ctx->b = b;
    const int st = halo_exchange(ctx, xr.d(), &Qin, &off);
    ctx->d_qext = keep_ext;
    ctx->qext_cap = keep_cap;
    ctx->d_sendbuf = keep_send;
    ctx->b = keep_b;
    if (st < 0) return st;
  }
  {
    const int st = apply_A(ctx, Qin, off, b, y.d(), nullptr, nullptr, nullptr);
    if (st < 0) return st;
  }
  HIPC(hipGetLastError());
  CHK(push_halo(ctx, xr.d(), b, y.d()));
  rowmajor_to_colmajor(y.d(), ctx->nloc, b, x.d(), ctx->stream);
  HIPC(hipMemcpyAsync(Y, x.p, ctx->nloc * b * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  return RBL_OK;
}

int rbl_start(rbl_ctx* ctx, int b, int max_blocks, int basis_bits, const double* omega,
              uint64_t seed) {
  if (!ctx) return RBL_ERR_INVALID;
  if (!has_matrix(ctx)) return fail(ctx, RBL_ERR_STATE, "rbl_start: no matrix");
  if (b < 1 || b > RBL_MAX_BLOCK)
    return fail(ctx, RBL_ERR_INVALID, "block size must be in [1," + std::to_string(RBL_MAX_BLOCK) + "]");
  if (max_blocks < 1) return fail(ctx, RBL_ERR_INVALID, "max_blocks must be >= 1");
  if (basis_bits != 64 && basis_bits != 32)
    return fail(ctx, RBL_ERR_INVALID, "basis_bits must be 64 or 32");
  HIPC(hipSetDevice(ctx->device));
  HIPC(hipStreamSynchronize(ctx->stream));
  // a repeated run with the same shape reuses the HBM plan (allocating ~100 GB of basis
  // per run costs more than the run itself at n = 1e7)
  // device slots of the basis (RBL_OPT_DEVICE_BLOCKS; RBL_gpu.jl:95-104 gpu_buffer_size)
  int dev_slots = max_blocks + 1;
  // the shape of the current plan matches: the automatic plan (G = -1) keeps its slot count
  // instead of re-deriving it from the free memory its own buffers now occupy — re-planning
  // frees and re-allocates the basis and unpins / re-pins every host spill slot (C5: ~40 s per
  // run on the host, hipHostMalloc / hipHostFree of ~80 GB)
  const bool same_shape = (ctx->d_basis || ctx->d_basis32) && ctx->b == b &&
                          ctx->max_blocks == max_blocks && ctx->slot == ctx->nloc * b &&
                          ctx->basis_bits == basis_bits;
  const int cur_slots = ctx->resident == INT32_MAX ? ctx->max_blocks + 1 : ctx->resident + 2;
  if (ctx->dev_blocks_opt < 0 && same_shape && ctx->auto_planned) {
    dev_slots = cur_slots;
  } else if (ctx->dev_blocks_opt != 0) {
    int g = ctx->dev_blocks_opt;
    if (g < 0) {
      size_t fr = 0, tot = 0;
      HIPC(hipMemGetInfo(&fr, &tot));
      // the basis is typed FLOAT (RBL_gpu.jl:59-81, 95-104): slots of n_local x b x s bytes
      const double blk64 = (double)std::max<int64_t>(ctx->nloc, 1) * b * 8.0;
      const double blk = blk64 * (basis_bits == 64 ? 1.0 : 0.5);
      // what the run needs beside the basis: U, T, the halo copy, staging, the fp64 working
      // block of the fp32 path, ~slab; a run already planned frees its buffers first
      const double mine = ctx->d_basis ? (double)(ctx->resident == INT32_MAX ? ctx->max_blocks + 1 : ctx->resident + 2) * blk64
                        : ctx->d_basis32 ? (double)(ctx->resident == INT32_MAX ? ctx->max_blocks + 1 : ctx->resident + 2) * blk64 * 0.5
                        : 0.0;
      // U, T (+ the halo buffer on several ranks; + the fp32 path's fp64 Q_i, and Q_{i-1}
      // when the SpMM cannot read fp32), one staging block, the Gram slab
      const double work = 2.0 + (ctx->nranks > 1 ? 1.0 : 0.0) +
                          (basis_bits == 32 ? 1.0 + (direct32_ok(ctx, b) ? 0.0 : 1.0) : 0.0);
      const double other = work * blk64 + blk + 8.0 * (double)gram_slab_elems(ctx, b, max_blocks, basis_bits);
      g = (int)std::max(3.0, std::floor((0.8 * ((double)fr + mine) - other) / blk));
    }
    dev_slots = std::min(dev_slots, std::max(3, g));
  }
  const bool reuse = same_shape && cur_slots == dev_slots;
  ctx->nlock = 0;  // a new problem: no locked vectors
  ctx->cloc_step = 0;
  ctx->step_flags.clear();
  // the allocations below fail alone on one rank (its HBM): every rank then learns of it before
  // the collectives of the start, and all return the error, instead of the peers waiting in the
  // halo exchange for a rank that has left
  const int alloc_st = [&]() -> int {
  if (reuse) {
    ctx->nblocks = 0;
    if (ctx->cstream) HIPC(hipStreamSynchronize(ctx->cstream));
    ctx->d2h_pending[0] = ctx->d2h_pending[1] = false;
    HIPC(hipMemsetAsync(ctx->d_flags, 0, 4 * sizeof(int), ctx->stream));
  } else {
  free_run(ctx);
  ctx->b = b;
  ctx->max_blocks = max_blocks;
  ctx->slot = ctx->nloc * b;
  const int64_t nl = std::max<int64_t>(ctx->nloc, 1);
  ctx->basis_bits = basis_bits;
  ctx->auto_planned = ctx->dev_blocks_opt < 0;
  if (basis_bits == 64) {
    HIPC(hipMalloc(&ctx->d_basis, (size_t)dev_slots * nl * b * sizeof(double)));
    if (dev_slots < max_blocks + 1) {  // host spill: pinned slots for blocks resident..max_blocks
      ctx->resident = dev_slots - 2;
      // non-coherent pinned pages: the DMA engines stream them at PCIe rate both ways
      ctx->h_spill.assign(max_blocks + 1 - ctx->resident, nullptr);
      HIPC(hipMalloc(&ctx->d_stage, (size_t)nl * b * sizeof(double)));
      if (!ctx->cstream) {
        HIPC(hipStreamCreateWithFlags(&ctx->cstream, hipStreamNonBlocking));
        HIPC(hipEventCreateWithFlags(&ctx->ev_fin, hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&ctx->ev_d2h[0], hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&ctx->ev_d2h[1], hipEventDisableTiming));
      }
    }
  } else {
    // + kRowPad32 zeroed pad rows, and every slot zeroed once: the fp32 Gram kernel's shifted
    // chunks may read rows past a tiny slice (reorth32.hip), which must be finite
    const size_t bytes32 = ((size_t)dev_slots * nl + kRowPad32) * b * sizeof(float);
    HIPC(hipMalloc(&ctx->d_basis32, bytes32));
    HIPC(hipMemsetAsync(ctx->d_basis32, 0, bytes32, ctx->stream));
    if (dev_slots < max_blocks + 1) {  // host spill of the FLOAT basis (RBL_gpu.jl:59-81)
      ctx->resident = dev_slots - 2;
      ctx->h_spill.assign(max_blocks + 1 - ctx->resident, nullptr);
      // + kRowPad32 zero rows like the slots (the Gram's shifted chunks)
      HIPC(hipMalloc(&ctx->d_stage32, ((size_t)nl + kRowPad32) * b * sizeof(float)));
      HIPC(hipMemsetAsync(ctx->d_stage32, 0, ((size_t)nl + kRowPad32) * b * sizeof(float), ctx->stream));
      if (!ctx->cstream) {
        HIPC(hipStreamCreateWithFlags(&ctx->cstream, hipStreamNonBlocking));
        HIPC(hipEventCreateWithFlags(&ctx->ev_fin, hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&ctx->ev_d2h[0], hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&ctx->ev_d2h[1], hipEventDisableTiming));
      }
    }
    HIPC(hipMalloc(&ctx->d_Qi64, (nl + kRowPad) * b * sizeof(double)));
    // the widened Q_{i-1}: only when the SpMM cannot read the fp32 blocks directly
    if (!direct32_ok(ctx, b)) HIPC(hipMalloc(&ctx->d_Qm64, (nl + kRowPad) * b * sizeof(double)));
  }
  HIPC(hipMalloc(&ctx->d_U, (nl + kRowPad) * b * sizeof(double)));
  ctx->T_cols = b;
  HIPC(hipMalloc(&ctx->d_T, nl * b * sizeof(double)));
  if (ctx->nranks > 1) {
    CHK(ensure_qext(ctx, b, ctx->stream));
    if (ctx->ghost)
      HIPC(hipMalloc(&ctx->d_sendbuf, std::max<int64_t>(ctx->n_send, 1) * b * sizeof(double)));
  }
  const size_t slab = gram_slab_elems(ctx, b, max_blocks, basis_bits);
  ctx->slab_elems = slab;
  HIPC(hipMalloc(&ctx->d_slab, slab * sizeof(double)));
  ctx->C_elems = (size_t)std::max(1, max_blocks) * b * 2 * b;
  HIPC(hipMalloc(&ctx->d_C, ctx->C_elems * sizeof(double)));
  HIPC(hipMalloc(&ctx->d_small, (size_t)S_NSMALL * b * b * sizeof(double)));
  HIPC(hipMalloc(&ctx->d_flags, 4 * sizeof(int)));
  HIPC(hipMemset(ctx->d_flags, 0, 4 * sizeof(int)));
  {
#ifdef RBL_VARIANTS
    const char* e = std::getenv("RBL_STASH_COPY");  // A/B: 1 = device record + D2H copy
    ctx->stash_direct = !(e && std::atoi(e) == 1);
#else
    ctx->stash_direct = true;
#endif
    const unsigned hf = ctx->stash_direct ? (hipHostMallocMapped | hipHostMallocCoherent) : hipHostMallocDefault;
    HIPC(hipHostMalloc(&ctx->h_pin, stash_rec(b) * sizeof(double), hf));
    HIPC(hipHostMalloc(&ctx->h_hist, (size_t)(max_blocks + 2) * stash_rec(b) * sizeof(double), hf));
    if ((size_t)ctx->nloc * b * sizeof(double) >= 4 * kD2HPiece && !d2h_direct()) {
      CHK(ensure_d2h_slots(ctx));
      CHK(ensure_ritz_stream(ctx));
    }
    if (ctx->stash_direct) {
      HIPC(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->dv_pin), ctx->h_pin, 0));
      HIPC(hipHostGetDevicePointer(reinterpret_cast<void**>(&ctx->dv_hist), ctx->h_hist, 0));
    } else {
      HIPC(hipMalloc(&ctx->d_stash, stash_rec(b) * sizeof(double)));
    }
  }
  }
  // the push/pull split's partial-row buffers (sized by the matrix held, so also on a reused
  // plan): allocated here, inside the vote, not lazily in the first push exchange — a rank
  // failing there would leave its peers waiting in that exchange
  if (ctx->push && ctx->nranks > 1 && use_ghost(ctx, b)) {  // push_on() once this b exchanges
    const char* inj = std::getenv("RBL_FAULT_PUSH_ALLOC");  // fault injection for the vote's test
    if (inj && *inj && std::atoi(inj) == ctx->rank)
      return fail(ctx, RBL_ERR_OOM, "rbl_start: push buffers (injected by RBL_FAULT_PUSH_ALLOC)");
    CHK(ensure_push(ctx, b));
  }
  return RBL_OK;
  }();
  if (ctx->nranks > 1) {
    const int64_t mine = alloc_st;
    std::vector<int64_t> all(ctx->nranks);
    COMMC(ctx->comm->allgather_host(&mine, all.data(), 1, ctx->stream, &ctx->err));
    int bad = -1;
    for (int q = 0; q < ctx->nranks && bad < 0; ++q)
      if (all[q] != RBL_OK) bad = q;
    if (bad >= 0) {
      (void)hipGetLastError();  // the failed hipMalloc's error must not surface in a later check
      free_run(ctx);  // (a later start re-plans from scratch)
      if (alloc_st != RBL_OK) return alloc_st;
      return fail(ctx, (int)all[bad], "rbl_start: rank " + std::to_string(bad) +
                                          " could not allocate its run buffers");
    }
  } else if (alloc_st != RBL_OK) {
    (void)hipGetLastError();
    return alloc_st;
  }

  // Omega (row-major) in d_T
  if (omega) {
    double* d_tmp = ctx->d_U;  // free until A * Omega
    HIPC(hipMemcpyAsync(d_tmp, omega, ctx->nloc * b * sizeof(double), hipMemcpyHostToDevice,
                        ctx->stream));
    colmajor_to_rowmajor(d_tmp, ctx->nloc, b, ctx->d_T, ctx->stream);
  } else {
    randn_block(ctx->d_T, ctx->nloc, b, ctx->r0, seed, ctx->stream,
                ctx->relabeled ? &ctx->relabel_perm : nullptr);
  }
  // Q_1 = qr(A * Omega).Q   (RBL_gpu.jl:213-214)
  const double* Qin = nullptr;
  int64_t off = 0;
  CHK(halo_exchange(ctx, ctx->d_T, &Qin, &off));
  {
    StageScope t(ctx, RBL_STAGE_AQ);
    CHK(apply_A(ctx, Qin, off, b, ctx->d_U, nullptr, nullptr, nullptr));
    HIPC(hipGetLastError());
  }
  CHK(push_halo(ctx, ctx->d_T, b, ctx->d_U));
  if (basis_bits == 64) {
    CHK(tsqr(ctx, ctx->d_U, slotp(ctx, 0)));
  } else {  // step 1 multiplies the unrounded fp64 Q_1 (RBL_gpu.jl:142, 152); the basis holds fp32
    CHK(tsqr(ctx, ctx->d_U, ctx->d_Qi64));
    cvt_f64_to_f32(ctx->d_Qi64, slotp32(ctx, 0), ctx->nloc * b, ctx->stream);
  }
  HIPC(hipStreamSynchronize(ctx->stream));
  harvest_timers(ctx);
  int flags[4];
  HIPC(hipMemcpy(flags, ctx->d_flags, sizeof(flags), hipMemcpyDeviceToHost));
  if (flags[2]) return fail(ctx, RBL_ERR_NUMERIC, "QR breakdown in rbl_start");
  ctx->nblocks = 1;
  ctx->fetched = 1;
  return RBL_OK;
}

namespace {
int step_impl(rbl_ctx* ctx, int i, int part_reorth, double* A_out, double* B_out, bool async);
}
int rbl_step(rbl_ctx* ctx, int i, int part_reorth, double* A_out, double* B_out) {
  if (ctx && ctx->fetched < ctx->nblocks)
    return fail(ctx, RBL_ERR_STATE, "rbl_step: rbl_fetch the asynchronous steps first");
  const int rc = step_impl(ctx, i, part_reorth, A_out, B_out, false);
  if (ctx && rc >= 0) ctx->fetched = ctx->nblocks;
  return rc;
}
int rbl_step_async(rbl_ctx* ctx, int i, int part_reorth) {
  return step_impl(ctx, i, part_reorth, nullptr, nullptr, true);
}
int rbl_fetch(rbl_ctx* ctx, int i0, int i1, double* A_out, double* B_out, int* status_out) {
  if (!ctx) return RBL_ERR_INVALID;
  if (i0 != ctx->fetched || i1 < i0 || i1 > ctx->nblocks)
    return fail(ctx, RBL_ERR_INVALID, "rbl_fetch: [i0, i1) must start at the first unfetched step");
  HIPC(hipSetDevice(ctx->device));
  // steps enqueued after i1 - 1 (speculatively, while the host works on the T band) keep running
  const int last = i1 - 1;
  if (last >= 1 && last < (int)ctx->step_ev.size() && ctx->step_ev[last])
    HIPC(hipEventSynchronize(ctx->step_ev[last]));
  else
    HIPC(hipStreamSynchronize(ctx->stream));
  harvest_timers(ctx);
  const int b = ctx->b;
  int rc = RBL_OK;
  for (int j = i0; j < i1; ++j) {
    const double* h = ctx->h_hist + (size_t)j * stash_rec(b);
    const int* fl = reinterpret_cast<const int*>(h + 2 * b * b);
    double* A = A_out ? A_out + (size_t)(j - i0) * b * b : nullptr;
    double* B = B_out ? B_out + (size_t)(j - i0) * b * b : nullptr;
    for (int r = 0; r < b; ++r)
      for (int c = 0; c < b; ++c) {
        if (A) A[c * b + r] = h[r * b + c];
        if (B) B[c * b + r] = h[b * b + r * b + c];
      }
    const int st = fl[2] ? RBL_ERR_NUMERIC : fl[3] ? RBL_WARN_QR_SHIFTED : RBL_OK;
    if (status_out) status_out[j - i0] = st;
    if (st == RBL_ERR_NUMERIC && rc >= 0) rc = fail(ctx, RBL_ERR_NUMERIC, "QR breakdown (shifted CholQR failed)");
  }
  ctx->fetched = i1;
  return rc;
}
namespace {
int step_impl(rbl_ctx* ctx, int i, int part_reorth, double* A_out, double* B_out, bool async) {
  if (!ctx) return RBL_ERR_INVALID;
  if ((!ctx->d_basis && !ctx->d_basis32) || ctx->nblocks < 1) return fail(ctx, RBL_ERR_STATE, "rbl_step before rbl_start");
  if (i != ctx->nblocks) return fail(ctx, RBL_ERR_STATE, "rbl_step: i must equal the current block count");
  if (i > ctx->max_blocks) return fail(ctx, RBL_ERR_STATE, "rbl_step: basis full (max_blocks)");
  HIPC(hipSetDevice(ctx->device));
  const int b = ctx->b;
  const bool f32 = ctx->basis_bits == 32;
  if (!ctx->flags_clean) HIPC(hipMemsetAsync(ctx->d_flags, 0, 4 * sizeof(int), ctx->stream));
  ctx->flags_clean = false;  // until this step's k_stash has run
  if (f32 && (part_reorth & 2))
    return fail(ctx, RBL_ERR_INVALID, "rbl_step: locked-vector reorth needs the fp64 basis");
  // fp32 basis with the band-tile SpMM: A Q_i (after an fp32 halo exchange) and the 3-term
  // update read the fp32 blocks and widen them on load — bit for bit the widened copies
  // (RBL_gpu.jl:173-174), without the two conversion passes.  Step 1 multiplies the unrounded
  // fp64 Q_1 of rbl_start.
  const bool direct32 = f32 && i >= 2 && direct32_ok(ctx, b);
  if (f32 && !direct32) CHK(ensure_qm64(ctx));
  double* Qi = f32 ? ctx->d_Qi64 : slotp(ctx, i - 1);
  double* Qm = i >= 2 ? (f32 ? ctx->d_Qm64 : slotp(ctx, i - 2)) : nullptr;
  float* Qi32 = f32 ? slotp32(ctx, i - 1) : nullptr;
  float* Qm32 = f32 && i >= 2 ? slotp32(ctx, i - 2) : nullptr;
  if (f32) {
    // FLOAT = Float32: partial and local reorth on the fp32 blocks, then the
    // current / previous block widened to fp64 (RBL_gpu.jl:164-174)
    if ((part_reorth & 1) && i >= 3) {
      StageScope t(ctx, RBL_STAGE_PART_REORTH);
      const int nW = i - 2;
      const int nres = std::min(nW, ctx->resident);  // HBM-resident part of W
      if (ctx->reorth_order == 0) {
        CHK(gram32(ctx, slotp32(ctx, 0), nres, Qi32, Qm32, 2, ctx->d_C));
        CHK(upd32(ctx, slotp32(ctx, 0), nres, ctx->d_C, 2 * b, Qi32, Qm32, 2));
      } else {
        for (int j = 0; j < nres; ++j) {
          CHK(gram32(ctx, slotp32(ctx, j), 1, Qi32, Qm32, 2, ctx->d_C));
          CHK(upd32(ctx, slotp32(ctx, j), 1, ctx->d_C, 2 * b, Qi32, Qm32, 2));
        }
      }
      // spilled fp32 blocks streamed back in ascending j (RBL_gpu.jl:65-68 with FLOAT)
      for (int j = nres; j < nW; ++j) {
        int st = 0;
        const float* Wj = block_dev32(ctx, j, i, &st);
        if (st) return fail(ctx, st, "partial reorth: H2D of a spilled block failed");
        CHK(gram32(ctx, Wj, 1, Qi32, Qm32, 2, ctx->d_C));
        CHK(upd32(ctx, Wj, 1, ctx->d_C, 2 * b, Qi32, Qm32, 2));
      }
    }
    // host spill: block i-2 is final (RBL_gpu.jl:76) — copied out on the side stream; the
    // QR of this step, which rewrites its working slot, waits for the copy
    if (spilled(ctx) && i >= 2 && i - 2 >= ctx->resident) {
      HIPC(hipEventRecord(ctx->ev_fin, ctx->stream));
      HIPC(hipStreamWaitEvent(ctx->cstream, ctx->ev_fin, 0));
      CHK(spill_slot(ctx, i - 2, sizeof(float)));
      HIPC(hipMemcpyAsync(ctx->h_spill[i - 2 - ctx->resident], Qm32,
                          ctx->slot * sizeof(float), hipMemcpyDeviceToHost, ctx->cstream));
      HIPC(hipEventRecord(ctx->ev_d2h[i & 1], ctx->cstream));
      ctx->d2h_pending[i & 1] = true;
    }
    if (i >= 2) {
      StageScope t(ctx, RBL_STAGE_LOC_REORTH);
      CHK(gram32(ctx, Qm32, 1, Qi32, nullptr, 1, ctx->d_C));
      CHK(upd32(ctx, Qm32, 1, ctx->d_C, b, Qi32, nullptr, 1));
      if (!direct32) {
        cvt_f32_to_f64(Qi32, ctx->d_Qi64, ctx->nloc * b, ctx->stream);
        cvt_f32_to_f64(Qm32, ctx->d_Qm64, ctx->nloc * b, ctx->stream);
      }
      HIPC(hipGetLastError());
    }
  }

  // partial reorth of Q_i and Q_{i-1} against Q_1..Q_{i-2}   (RBL_gpu.jl:164-166, 59-81),
  // preceded (flag bit 1, restarted variants) by the reorth against the locked vectors
  if (!f32) CHK(reorth_pair(ctx, i, part_reorth));
  // host spill: block i-2 is final now (the hybrid buffer's `copyto!(Q[i-1], Qg1)`,
  // RBL_gpu.jl:76): copy it out on the side stream while the step goes on; its working slot
  // is rewritten by this step's QR, which waits for the copy
  if (!f32 && spilled(ctx) && i >= 2 && i - 2 >= ctx->resident) {
    HIPC(hipEventRecord(ctx->ev_fin, ctx->stream));
    HIPC(hipStreamWaitEvent(ctx->cstream, ctx->ev_fin, 0));
    CHK(spill_slot(ctx, i - 2, sizeof(double)));
    HIPC(hipMemcpyAsync(ctx->h_spill[i - 2 - ctx->resident], slotp(ctx, i - 2),
                        ctx->slot * sizeof(double), hipMemcpyDeviceToHost, ctx->cstream));
    HIPC(hipEventRecord(ctx->ev_d2h[i & 1], ctx->cstream));
    ctx->d2h_pending[i & 1] = true;
  }
  // local reorth: Q_i -= Q_{i-1} (Q_{i-1}^T Q_i), one projection (RBL_gpu.jl:83-93, P1)
  const bool fused = rowgram_ok(b);
  // Q_i / Q_{i-1} change before the local reorth of this step iff it runs a partial or
  // locked-vector reorth; otherwise the Gram formed by the previous step's QR is current
  auto modifies = [&](int step, int flags) {
    return ((flags & 1) && step >= 3) || ((flags & 2) && ctx->nlock > 0);
  };
  if ((int)ctx->step_flags.size() <= i) ctx->step_flags.resize(i + 1, 0);
  ctx->step_flags[i] = part_reorth;
  // fuse bit 2: the update itself rides on the SpMM below, which stages Q_i's rows corrected
  // (fp64 basis, band tiles at b = 32; no collective depends on the choice)
  const bool lfuse = !f32 && i >= 2 && (ctx->fuse & 4) && fused && !ctx->dense && ctx->nloc > 0 &&
                     rbl_spmm_kernel_for(ctx, b) == 5 && spmm_bt_locfix_ok(csr(ctx), b);
  const double* Cloc = nullptr;
  int64_t lf_lo = 0, lf_hi = ctx->nloc;
  if (!f32 && i >= 2) {
    StageScope t(ctx, RBL_STAGE_LOC_REORTH);
    const bool have = ctx->cloc_step == i && (ctx->cloc_final || !modifies(i, part_reorth));
    const double* C = have ? smallp(ctx, S_CLOC) : ctx->d_C;
    if (!have) {
      CHK(gram(ctx, run1(Qm, b), pan1(Qi, b), ctx->d_C, nullptr));
      ctx->path_stats[RBL_PATH_LOC_GRAM] += 1;
    }
    if (lfuse) {
      Cloc = C;
      if (ctx->nranks > 1) {  // the rows the neighbours receive: corrected before the exchange
        const int64_t H = spmm_bt_halfwidth(csr(ctx));
        lf_lo = std::min<int64_t>(H, ctx->nloc);
        lf_hi = std::max<int64_t>(lf_lo, ctx->nloc - H);
        spmm_bt_locfix_edges(csr(ctx), Qi, Qm, C, 0, lf_lo, lf_hi, ctx->nloc, ctx->stream);
        HIPC(hipGetLastError());
        ctx->path_stats[RBL_PATH_LOCFIX_EDGES] += 1;
      }
    } else if (fused) {
      CHK(rowop(ctx, Qm, C, Qi, -1.0, 1.0, nullptr, nullptr));
      ctx->path_stats[RBL_PATH_LOC_SEPARATE] += 1;
    } else {
      CHK(tsmm_checked(ctx, run1(Qm, b), C, b, pan1(Qi, b), -1.0, 1.0, nullptr));
      ctx->path_stats[RBL_PATH_LOC_SEPARATE] += 1;
    }
  }
  ctx->cloc_step = 0;
  ctx->cloc_final = false;
  // U = A Q_i - Q_{i-1} B_i^T   (RBL_gpu.jl:176-177)
  int ai_parts = 0;
  bool pushed = false;  // the push/pull split's partials sent on the side stream
  {
    const double* Qin = nullptr;
    const float* Qin32 = nullptr;
    int64_t off = 0;
    // several ranks with the band-tile kernel: the halo buffer takes only the neighbours'
    // rows; the kernel reads the own rows from the block (no per-step local copy)
    const int kid = rbl_spmm_kernel_for(ctx, b);
    const bool seg_split = !direct32 && kid == 6 && ctx->seg_split;
    const bool split = ctx->nranks > 1 && !ctx->dense &&
                       (direct32 || kid == 5 || seg_split) && ctx->split_halo;
    // unbanded A on several ranks (the halo is most of Q_i): the exchange runs on a side
    // stream while the SpMM's own-column tier runs; the halo tier waits for it
    // (RBL_OPT_HALO_OVERLAP; the same sums in the same order either way)
    const bool overlap = split && seg_split && ctx->halo_overlap;
    hipEvent_t halo_ev = nullptr;
    if (overlap) {
      if (!ctx->hstream) {
        HIPC(hipStreamCreateWithFlags(&ctx->hstream, hipStreamNonBlocking));
        HIPC(hipEventCreateWithFlags(&ctx->ev_qready, hipEventDisableTiming));
        HIPC(hipEventCreateWithFlags(&ctx->ev_halo, hipEventDisableTiming));
      }
      HIPC(hipEventRecord(ctx->ev_qready, ctx->stream));  // Q_i final (local reorth done)
      HIPC(hipStreamWaitEvent(ctx->hstream, ctx->ev_qready, 0));
      CHK(halo_exchange(ctx, Qi, &Qin, &off, false, ctx->hstream));
      HIPC(hipEventRecord(ctx->ev_halo, ctx->hstream));
      halo_ev = ctx->ev_halo;
      if (push_on(ctx)) {  // the partials go out behind the pulled rows, before the SpMM
        if (!ctx->ev_push_ready) {
          HIPC(hipEventCreateWithFlags(&ctx->ev_push_ready, hipEventDisableTiming));
          HIPC(hipEventCreateWithFlags(&ctx->ev_push_done, hipEventDisableTiming));
        }
        CHK(push_products(ctx, Qi, b, ctx->stream));
        HIPC(hipEventRecord(ctx->ev_push_ready, ctx->stream));
        HIPC(hipStreamWaitEvent(ctx->hstream, ctx->ev_push_ready, 0));
        CHK(push_exchange(ctx, b, ctx->hstream));
        HIPC(hipEventRecord(ctx->ev_push_done, ctx->hstream));
        pushed = true;
      }
    } else if (direct32) {
      CHK(halo_exchange32(ctx, Qi32, &Qin32, &off, !split));
    } else {
      CHK(halo_exchange(ctx, Qi, &Qin, &off, !split));
    }
    StageScope t(ctx, RBL_STAGE_AQ);
    // the band kernel can also form the partials of A_i = Q_i^T U while U is in registers
    if (direct32) {
      CsrDev A = csr(ctx);
      if (split) {
        A.qloc = Qi32;
        A.loc_lo = ctx->r0;
        A.loc_hi = ctx->r0 + ctx->nloc;
      }
      if (!spmm_bt(A, nullptr, off, b, ctx->d_U, nullptr, smallp(ctx, S_BPREV), ctx->stream,
                   ctx->d_slab, &ai_parts, Qin32, Qm32))
        return fail(ctx, RBL_ERR_INVALID, "internal: fp32 band-tile SpMM not applicable");
    } else {
      ai_parts = apply_A(ctx, Qin, off, b, ctx->d_U, Qm, i >= 2 ? smallp(ctx, S_BPREV) : nullptr,
                         ctx->d_slab, split ? Qi : nullptr, Cloc, Qi, lf_lo, lf_hi, halo_ev);
    }
    if (ai_parts < 0) return ai_parts;
    HIPC(hipGetLastError());
    // the main stream's next collective must follow the side stream's exchange on every rank,
    // also where the SpMM never waited for it (a rank without rows returns from apply_A early)
    if (halo_ev) HIPC(hipStreamWaitEvent(ctx->stream, halo_ev, 0));
  }
  // the push/pull split: the received partials into U (A_i is formed after this, from all of U)
  if (pushed) {
    HIPC(hipStreamWaitEvent(ctx->stream, ctx->ev_push_done, 0));
    CHK(push_finish(ctx, ctx->d_U, b, ctx->stream));
  } else if (!direct32 && ai_parts == 0) {
    CHK(push_halo(ctx, Qi, b, ctx->d_U));
  }
  // A_i = Q_i^T U ; U -= Q_i A_i   (RBL_gpu.jl:178-179); fused: the update pass also forms
  // U^T U, CholQR's first Gram
  {
    StageScope t(ctx, RBL_STAGE_3TERM);
    if (ai_parts > 0) {
      reduce_slab(ctx->d_slab, ai_parts, (int64_t)b * b, smallp(ctx, S_AI), nullptr, ctx->stream);
      HIPC(hipGetLastError());
      CHK(allreduce(ctx, smallp(ctx, S_AI), (size_t)b * b));
    } else {
      CHK(gram(ctx, run1(Qi, b), pan1(ctx->d_U, b), smallp(ctx, S_AI), nullptr));
    }
    if (fused)
      CHK(rowop(ctx, Qi, smallp(ctx, S_AI), ctx->d_U, -1.0, 1.0, smallp(ctx, S_G), nullptr,
                direct32 ? Qi32 : nullptr));
    else
      CHK(tsmm_checked(ctx, run1(Qi, b), smallp(ctx, S_AI), b, pan1(ctx->d_U, b), -1.0, 1.0, nullptr));
  }
  // Q_{i+1} B_{i+1} = qr(U)   (RBL_gpu.jl:180-184)
  if (ctx->d2h_pending[i & 1]) {  // the working slot's previous block is on the host
    StageScope t(ctx, RBL_STAGE_SPILL_WAIT);  // the stream stalls here until that copy is done
    HIPC(hipStreamWaitEvent(ctx->stream, ctx->ev_d2h[i & 1], 0));
    ctx->d2h_pending[i & 1] = false;
  }
  if (!f32) {
    // the next step's local-reorth Gram Q_i^T Q_{i+1} rides on this QR when that step is
    // expected to run no partial reorth (the schedule repeats with period 2 in RBL_gpu.jl:164,
    // so step i + 1 is guessed from step i - 1; a wrong guess costs one pass, never bits)
    const int guess = i >= 2 ? ctx->step_flags[i - 1] : 0;
    const bool zfuse = fused && (ctx->fuse & 3) == 3 && !modifies(i + 1, guess) && i + 1 <= ctx->max_blocks;
    CHK(tsqr(ctx, ctx->d_U, slotp(ctx, i), fused, nullptr, zfuse ? Qi : nullptr));
    if (zfuse) {
      ctx->cloc_step = i + 1;
      ctx->cloc_final = false;
    }
  } else {  // Qg = FLOAT(Qg_d) (RBL_gpu.jl:182): the new block enters the basis rounded to fp32
    CHK(tsqr(ctx, ctx->d_U, ctx->d_Qi64, fused, slotp32(ctx, i)));
  }
  // B_prev = R_tot, and A_i, R_tot, flags as one record: written to the host by k_stash itself
  // (or one D2H copy of the device record, RBL_STASH_COPY=1)
  const size_t rec = stash_rec(b);
  double* rec_dev = !ctx->stash_direct ? ctx->d_stash
                    : async            ? ctx->dv_hist + (size_t)i * rec
                                       : ctx->dv_pin;
  stash_step(smallp(ctx, S_AI), smallp(ctx, S_RTOT), smallp(ctx, S_BPREV), ctx->d_flags, rec_dev,
             b, ctx->stream);
  ctx->flags_clean = true;
  if (async) {  // stash A_i, R_tot and the flags for rbl_fetch; no host round trip
    if (!ctx->stash_direct)
      HIPC(hipMemcpyAsync(ctx->h_hist + (size_t)i * rec, ctx->d_stash, rec * sizeof(double),
                          hipMemcpyDeviceToHost, ctx->stream));
    if ((int)ctx->step_ev.size() <= i) ctx->step_ev.resize(i + 1, nullptr);
    if (!ctx->step_ev[i]) HIPC(hipEventCreateWithFlags(&ctx->step_ev[i], hipEventDisableTiming));
    HIPC(hipEventRecord(ctx->step_ev[i], ctx->stream));
    HIPC(hipGetLastError());
    ctx->nblocks = i + 1;
    return RBL_OK;
  }
  if (!ctx->stash_direct)
    HIPC(hipMemcpyAsync(ctx->h_pin, ctx->d_stash, rec * sizeof(double), hipMemcpyDeviceToHost, ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  int flags[4];
  memcpy(flags, ctx->h_pin + 2 * b * b, sizeof(flags));
  harvest_timers(ctx);
  // row-major device -> column-major host
  for (int r = 0; r < b; ++r)
    for (int c = 0; c < b; ++c) {
      if (A_out) A_out[c * b + r] = ctx->h_pin[r * b + c];
      if (B_out) B_out[c * b + r] = ctx->h_pin[b * b + r * b + c];
    }
  ctx->nblocks = i + 1;
  if (flags[2]) return fail(ctx, RBL_ERR_NUMERIC, "QR breakdown (shifted CholQR failed)");
  return flags[3] ? RBL_WARN_QR_SHIFTED : RBL_OK;
}
// Device -> pageable host copy of a large result (the Ritz vectors, RBL_gpu.jl:219 returns them
// on the host) through two pinned 64 MiB slots: the DMA of piece p runs while host threads copy
// piece p-1 out of the other slot into the caller's memory.  hipMemcpy into pageable memory goes
// through the runtime's own bounce buffer on one thread, well under the PCIe rate (§2: 49-56 GB/s
// pinned).  Every earlier piece's host copy has finished before its slot is refilled.
// RBL_D2H_DIRECT=1 restores the plain copy (A/B).
int d2h_staged(rbl_ctx* ctx, void* dst, const void* src, size_t bytes) {
  if (bytes < 4 * kD2HPiece || d2h_direct()) {
    HIPC(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, ctx->stream));
    return RBL_OK;
  }
  CHK(ensure_d2h_slots(ctx));
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const char* envt = std::getenv("RBL_D2H_THREADS");
  const int nthr = (int)std::min(envt ? std::max(1u, (unsigned)atoi(envt)) : 8u, hw);
  auto host_copy = [&](size_t p) {
    const size_t off = p * kD2HPiece, len = std::min(kD2HPiece, bytes - off);
    char* d = static_cast<char*>(dst) + off;
    const char* s = static_cast<const char*>(ctx->h_d2h[p & 1]);
    const size_t part = ((len + nthr - 1) / nthr + 4095) & ~size_t(4095);
    std::vector<std::thread> th;
    for (size_t o = part; o < len; o += part)
      th.emplace_back([=] { memcpy(d + o, s + o, std::min(part, len - o)); });
    memcpy(d, s, std::min(part, len));
    for (auto& t : th) t.join();
  };
  const size_t np = (bytes + kD2HPiece - 1) / kD2HPiece;
  for (size_t p = 0; p <= np; ++p) {
    if (p < np) {
      const size_t off = p * kD2HPiece;
      HIPC(hipMemcpyAsync(ctx->h_d2h[p & 1], static_cast<const char*>(src) + off,
                          std::min(kD2HPiece, bytes - off), hipMemcpyDeviceToHost, ctx->stream));
      HIPC(hipEventRecord(ctx->ev_d2h_slot[p & 1], ctx->stream));
    }
    if (p > 0) {
      HIPC(hipEventSynchronize(ctx->ev_d2h_slot[(p - 1) & 1]));
      host_copy(p - 1);
    }
  }
  return RBL_OK;
}

// The Ritz vectors in row pieces with the D2H behind them (rbl_ritz, one chunk of k <= b columns,
// every block resident — fp64, or fp32 where the fp32-input MFMA combination applies — and a
// result of >= 4 staging pieces).  V = [Q_1..Q_m] S and its
// transpose run in kRitzPieces row pieces on a side stream; the staged D2H stays on the context's
// stream, each 64 MiB staging piece issued once the host has seen the row pieces it covers
// finish, so the PCIe copy
// (1.6 GB at ~53 GB/s, 30 ms at C4a) overlaps the basis reads of the later pieces (5.5 ms at 8
// blocks, 17.6 ms at 28) instead of following all of them.  (Copies ordered behind the pieces by
// a device-side stream wait ran at half the PCIe rate in most calls, on either stream:
// profiles/r05_ritz_pipelined_trace_b29.log.)  Piece p (rows [r_p, r_{p+1})) is stored column-major
// with its own row count as leading dimension, so the pieces tile the column-major buffer
// contiguously; the host scatters each staged byte range into V_out's columns.  Every row of V is
// the same sum in the same order as in the one-pass form, so V is bit-identical
// (test_ritz_pipelined_matches_one_pass).  RBL_RITZ_SERIAL=1 restores the one-pass form.
constexpr int kRitzPieces = 8;
int ritz_pipelined(rbl_ctx* ctx, int nblocks, int k, int kcp, const double* d_S, double* pV,
                   double* pVcm, double* V_out) {
  const int b = ctx->b;
  const int64_t nl = ctx->nloc;
  const int64_t pr = (nl / kRitzPieces) & ~int64_t(63);  // rows per piece; the last takes the rest
  int64_t r0p[kRitzPieces + 1];
  for (int p = 0; p < kRitzPieces; ++p) r0p[p] = p * pr;
  r0p[kRitzPieces] = nl;
  CHK(ensure_d2h_slots(ctx));
  CHK(ensure_ritz_stream(ctx));
  HIPC(hipEventRecord(ctx->ev_ritz[kRitzPieces], ctx->stream));  // S is on the device
  HIPC(hipStreamWaitEvent(ctx->rstream, ctx->ev_ritz[kRitzPieces], 0));
  // on every exit, error paths included: the side stream's kernels write U / T and the run
  // scratch, so nothing may leave here with them still queued behind the context's back
  struct DrainSide {
    hipStream_t s;
    ~DrainSide() { (void)hipStreamSynchronize(s); }
  } drain{ctx->rstream};
  {
    StageScope t(ctx, RBL_STAGE_RITZ, ctx->rstream);
    for (int p = 0; p < kRitzPieces; ++p) {
      const int64_t r0 = r0p[p], m = r0p[p + 1] - r0;
      PanelRun X;
      X.stride = ctx->slot;
      X.count = nblocks;
      X.w = b;
      if (ctx->basis_bits == 64) {
        X.base = slotp(ctx, 0) + r0 * b;
        tsmm(m, X, d_S, kcp, pan1(pV + r0 * kcp, kcp), 1.0, 0.0, nullptr, ctx->rstream);
      } else {  // fp32 basis: the fp32-input MFMA form of combine_blocks32, widened on load
        X.base32 = slotp32(ctx, 0) + r0 * b;
        tsmm44_f32x(m, X, d_S, kcp, pan1(pV + r0 * kcp, kcp), 1.0, 0.0, ctx->rstream);
      }
      rowmajor_to_colmajor(pV + r0 * kcp, m, kcp, pVcm + r0 * kcp, ctx->rstream);
      HIPC(hipEventRecord(ctx->ev_ritz[p], ctx->rstream));
    }
  }
  HIPC(hipGetLastError());
  const char* src = reinterpret_cast<const char*>(pVcm);
  const size_t bytes = (size_t)nl * kcp * sizeof(double);
  auto piece_of = [&](size_t o) {  // the row piece holding byte o of the column-major buffer
    int p = 0;
    while (p + 1 < kRitzPieces && (size_t)r0p[p + 1] * kcp * sizeof(double) <= o) ++p;
    return p;
  };
  // device bytes [a, e) of staging piece q (slot q & 1) -> V_out's columns (padding column skipped)
  auto scatter = [&](size_t q, size_t a, size_t e) {
    const char* slot = static_cast<const char*>(ctx->h_d2h[q & 1]);
    const size_t base = q * kD2HPiece;
    for (size_t o = base + a; o < base + e;) {
      const int p = piece_of(o);
      const int64_t r0 = r0p[p], m = r0p[p + 1] - r0;
      const size_t colb = (size_t)m * sizeof(double);
      const size_t within = o - (size_t)r0 * kcp * sizeof(double);
      const size_t c = within / colb, inr = within % colb;
      const size_t run = std::min(base + e, o + (colb - inr));
      if ((int)c < k)
        memcpy(reinterpret_cast<char*>(V_out + (int64_t)c * nl + r0) + inr, slot + (o - base), run - o);
      o = run;
    }
  };
  const unsigned hw = std::max(1u, std::thread::hardware_concurrency());
  const char* envt = std::getenv("RBL_D2H_THREADS");
  const int nthr = (int)std::min(envt ? std::max(1u, (unsigned)atoi(envt)) : 8u, hw);
  const size_t nq = (bytes + kD2HPiece - 1) / kD2HPiece;
  int waited = -1;  // the last row piece the context's stream waits for
  for (size_t q = 0; q <= nq; ++q) {
    if (q < nq) {
      const size_t off = q * kD2HPiece, len = std::min(kD2HPiece, bytes - off);
      // the host waits for the pieces, so the copy carries no cross-stream dependency (copies
      // queued behind a hipStreamWaitEvent ran at half the PCIe rate, ~28 GB/s)
      for (const int pl = piece_of(off + len - 1); waited < pl;)
        HIPC(hipEventSynchronize(ctx->ev_ritz[++waited]));
      HIPC(hipMemcpyAsync(ctx->h_d2h[q & 1], src + off, len, hipMemcpyDeviceToHost, ctx->stream));
      HIPC(hipEventRecord(ctx->ev_d2h_slot[q & 1], ctx->stream));
    }
    if (q > 0) {
      const size_t pq = q - 1, len = std::min(kD2HPiece, bytes - pq * kD2HPiece);
      HIPC(hipEventSynchronize(ctx->ev_d2h_slot[pq & 1]));
      const size_t part = ((len + nthr - 1) / nthr + 4095) & ~size_t(4095);
      std::vector<std::thread> th;
      for (size_t o = part; o < len; o += part)
        th.emplace_back([=, &scatter] { scatter(pq, o, std::min(len, o + part)); });
      scatter(pq, 0, std::min(part, len));
      for (auto& t : th) t.join();
    }
  }
  // every piece has finished (the host waited for the last before its copy); later work on the
  // context's stream (the next run's steps reuse U and T) follows the side stream's kernels
  HIPC(hipStreamSynchronize(ctx->rstream));
  HIPC(hipStreamSynchronize(ctx->stream));
  return RBL_OK;
}
}  // namespace

int rbl_ritz(rbl_ctx* ctx, int nblocks, int k, const double* S, double* V_out) {
  if (!ctx || nblocks < 1 || k < 1 || !S) return fail(ctx, RBL_ERR_INVALID, "rbl_ritz: bad arguments");
  if (nblocks > ctx->nblocks) return fail(ctx, RBL_ERR_INVALID, "rbl_ritz: more blocks than computed");
  if (k > nblocks * ctx->b) return fail(ctx, RBL_ERR_INVALID, "rbl_ritz: k > nblocks*b");
  HIPC(hipSetDevice(ctx->device));
  const int b = ctx->b;
  const int64_t rows = (int64_t)nblocks * b;
  const int64_t nl = std::max<int64_t>(ctx->nloc, 1);
  // Ritz columns in chunks of <= 64 (one tsmm44 launch each), halved while a chunk's buffers
  // (S rows, V and its column-major copy) exceed 0.7 of free HBM — RBL_gpu.jl:24-27, 110-125
  // (`blocksize`).  Each chunk reads the basis once.
  size_t free_b = 0, total_b = 0;
  HIPC(hipMemGetInfo(&free_b, &total_b));
  int kc = std::min(k, 64);
  auto chunk_bytes = [&](int w) { return (double)((w + 1) & ~1) * (double)(rows + 2 * nl) * 8.0; };
  while (kc > 1 && chunk_bytes(kc) > 0.7 * (double)free_b) kc = (kc + 1) / 2;
  const int kcp = (kc + 1) & ~1;  // even panel width (16-B row stores), zero-padded column
  if (chunk_bytes(kc) > 0.7 * (double)free_b)
    return fail(ctx, RBL_ERR_OOM, "rbl_ritz: no room for one Ritz column");
  // RBL_RITZ_TRACE=1: host-side split of the call on stderr (diagnostics)
#ifdef RBL_VARIANTS
  const bool trace = std::getenv("RBL_RITZ_TRACE") != nullptr;
#else
  const bool trace = false;
#endif
  auto tnow = [] { return std::chrono::duration<double, std::milli>(
                       std::chrono::steady_clock::now().time_since_epoch()).count(); };
  const double t0 = trace ? tnow() : 0.0;
  double t_alloc = 0.0, t_comp = 0.0, t_d2h = 0.0;
  // the run's scratch blocks hold a chunk when it is at most b wide (k <= b: every chunk): U
  // (n_local x b) takes V, T the column-major copy, the coefficient buffer (max_blocks b x 2b)
  // the S rows — no 2 x n_local x kcp allocation per call (at C4a 3.2 GB, whose hipMalloc +
  // first touch cost up to ~20 ms of a time-to-k)
  DevBuf own_S, own_V, own_Vcm;
  double *pS = nullptr, *pV = nullptr, *pVcm = nullptr;
  if (kcp <= b && ctx->d_U && ctx->d_T && ctx->d_C && (size_t)rows * kcp <= ctx->C_elems) {
    pS = ctx->d_C;
    pV = ctx->d_U;
    pVcm = ctx->d_T;
  } else {
    HIPC(hipMalloc(&own_S.p, rows * kcp * sizeof(double)));
    HIPC(hipMalloc(&own_V.p, nl * kcp * sizeof(double)));
    HIPC(hipMalloc(&own_Vcm.p, nl * kcp * sizeof(double)));
    pS = own_S.d();
    pV = own_V.d();
    pVcm = own_Vcm.d();
  }
  if (trace) t_alloc = tnow() - t0;
  const bool pipelined = V_out && ctx->nloc > 0 && kc >= k && pV == ctx->d_U &&
                         (ctx->basis_bits == 64 || tsmm44_ok(b, kcp, kcp)) &&
                         nblocks <= ctx->resident && ctx->nloc >= 64 * kRitzPieces &&
                         (size_t)ctx->nloc * kcp * sizeof(double) >= 4 * kD2HPiece &&
                         !d2h_direct() && !ritz_serial();
  std::vector<double> srm((size_t)rows * kcp);
  if (pipelined) {
    for (int64_t r = 0; r < rows; ++r)
      for (int c = 0; c < kcp; ++c) srm[(size_t)r * kcp + c] = c < k ? S[(size_t)c * rows + r] : 0.0;
    HIPC(hipMemcpyAsync(pS, srm.data(), rows * kcp * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    ctx->path_stats[RBL_PATH_RITZ_PIECES] += 1;
    CHK(ritz_pipelined(ctx, nblocks, k, kcp, pS, pV, pVcm, V_out));
    harvest_timers(ctx);
    if (trace) fprintf(stderr, "rbl_ritz: pipelined, %d row pieces, total %.2f ms\n", kRitzPieces, tnow() - t0);
    return RBL_OK;
  }
  for (int c0 = 0; c0 < k; c0 += kc) {
    const int w = std::min(kc, k - c0);
    // the previous chunk's copy may still read srm (HIP does not promise a pageable source is
    // consumed when hipMemcpyAsync returns): wait for it before refilling
    HIPC(hipStreamSynchronize(ctx->stream));
    // S columns [c0, c0 + w) (column-major, ld = rows) -> row-major rows x kcp, zero-padded
    for (int64_t r = 0; r < rows; ++r)
      for (int c = 0; c < kcp; ++c) srm[(size_t)r * kcp + c] = c < w ? S[(size_t)(c0 + c) * rows + r] : 0.0;
    HIPC(hipMemcpyAsync(pS, srm.data(), rows * kcp * sizeof(double), hipMemcpyHostToDevice, ctx->stream));
    {
      StageScope t(ctx, RBL_STAGE_RITZ);
      if (ctx->basis_bits == 64) CHK(combine_blocks(ctx, nblocks, kcp, pS, pV));
      else CHK(combine_blocks32(ctx, nblocks, kcp, pS, pV));
    }
    if (ctx->nloc > 0) rowmajor_to_colmajor(pV, ctx->nloc, kcp, pVcm, ctx->stream);
    HIPC(hipGetLastError());
    double tc = 0.0;
    if (trace) {
      HIPC(hipStreamSynchronize(ctx->stream));
      tc = tnow();
      t_comp += tc - t0 - t_alloc - t_comp - t_d2h;
    }
    if (V_out && ctx->nloc > 0)
      CHK(d2h_staged(ctx, V_out + (size_t)c0 * ctx->nloc, pVcm, ctx->nloc * w * sizeof(double)));
    if (trace) {
      HIPC(hipStreamSynchronize(ctx->stream));
      t_d2h += tnow() - tc;
    }
  }
  HIPC(hipStreamSynchronize(ctx->stream));
  harvest_timers(ctx);
  if (trace)
    fprintf(stderr, "rbl_ritz: alloc %.2f ms, S + combine + transpose %.2f ms, D2H %.2f ms, total %.2f ms\n",
            t_alloc, t_comp, t_d2h, tnow() - t0);
  return RBL_OK;
}

int rbl_get_block(rbl_ctx* ctx, int j, double* Q_out) {
  if (!ctx || j < 1 || j > ctx->nblocks || !Q_out) return fail(ctx, RBL_ERR_INVALID, "rbl_get_block: bad block");
  HIPC(hipSetDevice(ctx->device));
  const int b = ctx->b;
  int st = 0;
  const double* src = ctx->basis_bits == 64 ? block_dev(ctx, j - 1, ctx->nblocks, &st) : nullptr;
  if (st) return fail(ctx, st, "rbl_get_block: H2D of a spilled block failed");
  if (ctx->basis_bits == 32) {  // fp32 slot, returned widened
    CHK(ensure_qm64(ctx));
    const float* s32 = block_dev32(ctx, j - 1, ctx->nblocks, &st);
    if (st) return fail(ctx, st, "rbl_get_block: H2D of a spilled block failed");
    cvt_f32_to_f64(s32, ctx->d_Qm64, ctx->nloc * b, ctx->stream);
    src = ctx->d_Qm64;
  }
  rowmajor_to_colmajor(src, ctx->nloc, b, ctx->d_T, ctx->stream);
  HIPC(hipMemcpyAsync(Q_out, ctx->d_T, ctx->nloc * b * sizeof(double), hipMemcpyDeviceToHost,
                      ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  return RBL_OK;
}

int rbl_num_blocks(rbl_ctx* ctx) { return ctx ? ctx->nblocks : 0; }

// ---- restarted variants (restarted.jl) -------------------------------------------------
int rbl_restart(rbl_ctx* ctx, int nblocks, const double* S) {
  if (ctx) ctx->cloc_step = 0;  // the basis changes outside the step
  if (!ctx || !S || nblocks < 1 || nblocks > ctx->nblocks)
    return fail(ctx, RBL_ERR_INVALID, "rbl_restart: bad arguments");
  if (!ctx->d_basis) return fail(ctx, RBL_ERR_STATE, "rbl_restart: needs an fp64 run (rbl_start)");
  if (spilled(ctx)) return fail(ctx, RBL_ERR_STATE, "rbl_restart: needs an HBM-resident basis");
  HIPC(hipSetDevice(ctx->device));
  const int b = ctx->b;
  CHK(basis_combine(ctx, nblocks, b, S, ctx->d_T));
  HIPC(hipMemcpyAsync(slotp(ctx, 0), ctx->d_T, ctx->nloc * b * sizeof(double),
                      hipMemcpyDeviceToDevice, ctx->stream));
  HIPC(hipMemsetAsync(ctx->d_flags, 0, 4 * sizeof(int), ctx->stream));
  HIPC(hipStreamSynchronize(ctx->stream));
  ctx->nblocks = 1;
  ctx->fetched = 1;
  return RBL_OK;
}

int rbl_lock(rbl_ctx* ctx, int nblocks, int nvec, const double* S) {
  if (ctx) ctx->cloc_step = 0;  // the basis changes outside the step
  if (!ctx || !S || nblocks < 1 || nblocks > ctx->nblocks || nvec < 0)
    return fail(ctx, RBL_ERR_INVALID, "rbl_lock: bad arguments");
  if (!ctx->d_basis) return fail(ctx, RBL_ERR_STATE, "rbl_lock: needs an fp64 run (rbl_start)");
  if (spilled(ctx)) return fail(ctx, RBL_ERR_STATE, "rbl_lock: needs an HBM-resident basis");
  if (nvec == 0) return RBL_OK;
  HIPC(hipSetDevice(ctx->device));
  const int64_t nl = std::max<int64_t>(ctx->nloc, 1);
  if (ctx->nlock + nvec > ctx->lock_cap) {
    const int cap = std::max(2 * ctx->lock_cap, ctx->nlock + nvec);
    double* d = nullptr;
    HIPC(hipMalloc(&d, (size_t)cap * nl * sizeof(double)));
    if (ctx->nlock)
      HIPC(hipMemcpyAsync(d, ctx->d_lock, (size_t)ctx->nlock * nl * sizeof(double),
                          hipMemcpyDeviceToDevice, ctx->stream));
    HIPC(hipStreamSynchronize(ctx->stream));
    hipFree(ctx->d_lock);
    ctx->d_lock = d;
    ctx->lock_cap = cap;
  }
  const int64_t rows = (int64_t)nblocks * ctx->b;
  for (int v = 0; v < nvec; ++v)
    CHK(basis_combine(ctx, nblocks, 1, S + v * rows, ctx->d_lock + (int64_t)(ctx->nlock + v) * nl));
  ctx->nlock += nvec;
  return RBL_OK;
}

int rbl_num_locked(rbl_ctx* ctx) { return ctx ? ctx->nlock : 0; }

int rbl_get_locked(rbl_ctx* ctx, double* V_out) {
  if (!ctx || !V_out) return fail(ctx, RBL_ERR_INVALID, "rbl_get_locked: bad arguments");
  if (ctx->nlock == 0) return RBL_OK;
  HIPC(hipSetDevice(ctx->device));
  const int64_t nl = std::max<int64_t>(ctx->nloc, 1);
  for (int j = 0; j < ctx->nlock; ++j)  // vector j is a contiguous column of length n_local
    HIPC(hipMemcpy(V_out + (int64_t)j * ctx->nloc, ctx->d_lock + (int64_t)j * nl,
                   ctx->nloc * sizeof(double), hipMemcpyDeviceToHost));
  return RBL_OK;
}

int rbl_reorth_last(rbl_ctx* ctx, int nblocks, int flags) {
  if (ctx) ctx->cloc_step = 0;  // the basis changes outside the step
  if (!ctx || nblocks < 1 || nblocks > ctx->nblocks)
    return fail(ctx, RBL_ERR_INVALID, "rbl_reorth_last: bad arguments");
  if (!ctx->d_basis) return fail(ctx, RBL_ERR_STATE, "rbl_reorth_last: needs an fp64 run");
  if (spilled(ctx)) return fail(ctx, RBL_ERR_STATE, "rbl_reorth_last: needs an HBM-resident basis");
  HIPC(hipSetDevice(ctx->device));
  CHK(reorth_pair(ctx, nblocks, flags));
  HIPC(hipStreamSynchronize(ctx->stream));
  harvest_timers(ctx);
  return RBL_OK;
}

int rbl_num_stages(void) { return RBL_NUM_STAGES; }
const char* rbl_stage_name(int stage) {
  return (stage >= 0 && stage < RBL_NUM_STAGES) ? kStageNames[stage] : "";
}
int rbl_timers(rbl_ctx* ctx, double* ms, int nstages) {
  if (!ctx || !ms) return RBL_ERR_INVALID;
  for (int s = 0; s < nstages && s < RBL_NUM_STAGES; ++s) ms[s] = ctx->stage_ms[s];
  return RBL_OK;
}
int rbl_allgather_host(rbl_ctx* ctx, const int64_t* mine, int64_t* all, int n) {
  if (!ctx || n < 0 || (n > 0 && (!mine || !all))) return fail(ctx, RBL_ERR_INVALID, "rbl_allgather_host: bad arguments");
  if (n == 0) return RBL_OK;
  HIPC(hipSetDevice(ctx->device));
  if (ctx->nranks == 1) {
    memcpy(all, mine, (size_t)n * sizeof(int64_t));
    return RBL_OK;
  }
  COMMC(ctx->comm->allgather_host(mine, all, (size_t)n, ctx->stream, &ctx->err));
  return RBL_OK;
}

int rbl_comm_stats(rbl_ctx* ctx, int64_t* out, int nstats, int reset) {
  if (!ctx || nstats < 0 || (nstats > 0 && !out)) return RBL_ERR_INVALID;
  for (int i = 0; i < nstats && i < RBL_COMM_NSTATS; ++i) out[i] = ctx->comm_stats[i];
  // the halo plan of the matrix held (not counters: reset leaves them)
  if (nstats > RBL_COMM_HALO_PUSH) out[RBL_COMM_HALO_PUSH] = ctx->push ? 1 : 0;
  if (nstats > RBL_COMM_PUSH_ROWS) out[RBL_COMM_PUSH_ROWS] = ctx->push_pred_rows;
  if (nstats > RBL_COMM_PULL_ROWS) out[RBL_COMM_PULL_ROWS] = ctx->pull_pred_rows;
  // the time in the collectives: host wall time in the calls, hipEvent spans on their streams
  const int64_t tm[4] = {ctx->comm_host_ns[0], ctx->comm_host_ns[1],
                         (int64_t)(ctx->comm_dev_ms[0] * 1e6), (int64_t)(ctx->comm_dev_ms[1] * 1e6)};
  for (int i = RBL_COMM_PULL_ROWS + 1; i < nstats; ++i)
    out[i] = i <= RBL_COMM_EXCHANGE_DEV_NS ? tm[i - RBL_COMM_ALLREDUCE_HOST_NS] : 0;
  if (reset) {
    for (int64_t& v : ctx->comm_stats) v = 0;
    ctx->comm_host_ns[0] = ctx->comm_host_ns[1] = 0;
    ctx->comm_dev_ms[0] = ctx->comm_dev_ms[1] = 0.0;
  }
  return RBL_OK;
}

int rbl_path_stats(rbl_ctx* ctx, int64_t* out, int nstats, int reset) {
  if (!ctx || nstats < 0 || (nstats > 0 && !out)) return RBL_ERR_INVALID;
  for (int i = 0; i < nstats; ++i) out[i] = i < RBL_PATH_NSTATS ? ctx->path_stats[i] : 0;
  if (reset)
    for (int64_t& v : ctx->path_stats) v = 0;
  return RBL_OK;
}

int rbl_reset_timers(rbl_ctx* ctx) {
  if (!ctx) return RBL_ERR_INVALID;
  for (double& v : ctx->stage_ms) v = 0.0;
  return RBL_OK;
}
int rbl_synchronize(rbl_ctx* ctx) {
  if (!ctx) return RBL_ERR_INVALID;
  HIPC(hipSetDevice(ctx->device));
  HIPC(hipStreamSynchronize(ctx->stream));
  harvest_timers(ctx);
  return RBL_OK;
}

}  // extern "C"
