/*
 * rbl_hip.h — C-ABI of librbl_hip.so, the MI355X (gfx950) Randomized Block Lanczos
 * inner loop.  Plain pointers and sizes only; no torch / HIP types cross this boundary.
 *
 * The reference (Iasonaspg/GPU-Randomized-Block-Lanczos) has no FFI layer: its "API" is
 * the Julia function pair RBL(A,k,b) (Julia/RBL.jl:119) / RBL_gpu(A,k,b)
 * (Julia/RBL_gpu.jl:205).  Its only native-call convention is the ccall into LAPACK at
 * Julia/common.jl:32-34 (ILP64 Ref{Int64} scalars, Ptr{Float64} column-major buffers).
 * This header follows that convention: int64 sizes, column-major dense buffers at the
 * boundary, caller-allocated outputs, every pointer borrowed only for the call.
 *
 * Each entry point below names the reference code it replaces.  The host loop that
 * replaces Julia/RBL_gpu.jl:162-194 (T_j assembly, dsbev, sort, convergence test —
 * Julia/common.jl:9-65) stays on the CPU and calls rbl_step() once per block step.
 *
 * Status codes: 0 ok, <0 error (rbl_last_error() has text), >0 warning.
 * Threading: one context per caller, not re-entrant; every entry point re-binds its
 * device, so callers may migrate between OS threads (Julia tasks).
 */
#ifndef RBL_HIP_H
#define RBL_HIP_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* 2: RBL_OPT_SPMM_KERNEL takes the kernel ids of rbl_spmm_kernel_for (5 band tiles, 6 segmented
 *    gather; version 1 took 4 / 5 for them) and rbl_create_shm was added.  A caller built
 *    against version 1 should check rbl_abi_version() before passing kernel ids. */
#define RBL_ABI_VERSION 2
/* Largest Krylov block size b (RBL_gpu(A, k, b) takes any b, RBL_gpu.jl:205; the reference's
 * scripts use b <= 8, the north star b = 32).  The MFMA fast paths cover b in {16, 32}. */
#define RBL_MAX_BLOCK 512

#define RBL_OK                  0
#define RBL_WARN_NOT_CONVERGED  1   /* host-side status for the P6 case */
#define RBL_WARN_QR_SHIFTED     2   /* rank-deficient block: shifted CholQR3 was used      */
#define RBL_ERR_INVALID        -1   /* bad argument / unsupported option                   */
#define RBL_ERR_HIP            -2   /* HIP runtime failure                                 */
#define RBL_ERR_OOM            -3   /* device allocation failed                            */
#define RBL_ERR_RCCL           -4   /* RCCL failure                                        */
#define RBL_ERR_STATE          -5   /* call out of order (e.g. step before start)          */
#define RBL_ERR_NUMERIC        -6   /* QR breakdown that the fallback could not repair     */

/* Timer stages; names match the reference's TimerOutputs labels (Julia/RBL_gpu.jl:152-187,219). */
#define RBL_STAGE_AQ          0   /* "AQ"            RBL_gpu.jl:152,176  SpMM + fused 3-term term */
#define RBL_STAGE_3TERM       1   /* "3-term"        RBL_gpu.jl:153-154,177-179                  */
#define RBL_STAGE_QR          2   /* "qr"            RBL_gpu.jl:155,180-184                      */
#define RBL_STAGE_PART_REORTH 3   /* "part reorth"   RBL_gpu.jl:165                               */
#define RBL_STAGE_LOC_REORTH  4   /* "loc reorth"    RBL_gpu.jl:167                               */
#define RBL_STAGE_RITZ        5   /* "Ritz vectors"  RBL_gpu.jl:219                               */
#define RBL_STAGE_COMM        6   /* halo exchange + all-reduce (no reference equivalent)         */
#define RBL_STAGE_SPILL_WAIT  7   /* "spill wait": host spill, the step's QR waiting for the D2H
                                   * copy-out of a finished block that shares its working slot  */
#define RBL_NUM_STAGES        8

/* Options for rbl_set_option(). */
#define RBL_OPT_TIMERS        0   /* 1: record per-stage hipEvents (adds event records);        */
                                  /*    2: only the "AQ" and "part reorth" stages (the kernels  */
                                  /*    the bench prices against their rooflines)               */
#define RBL_OPT_REORTH_ORDER  1   /* 0: block-CGS (batched, default); 1: ascending-j block MGS  */
                                  /*    exactly as RBL.jl:30-48 / RBL_gpu.jl:65-67               */
#define RBL_OPT_DEVICE_BLOCKS 3   /* Krylov blocks kept in HBM (the reference's hybrid buffer,
                                   * RBL_GPU.jl:24-27, 59-81, 95-132): 0 = all (default); -1 =
                                   * as many as fit in 80 % of free HBM (gpu_buffer_size);
                                   * G >= 3 = G slots: blocks 0..G-3 resident, the two newest
                                   * in two working slots, every older block in pinned host
                                   * memory, streamed back over PCIe for partial reorth and
                                   * Ritz.  fp64 or fp32 basis (the reference's buffer is typed
                                   * FLOAT, RBL_gpu.jl:59-81); set before rbl_start.            */
#define RBL_OPT_SPMM_KERNEL   2   /* 0: auto; otherwise the kernel id rbl_spmm_kernel_for reports:
                                   * 1 global-gather CSR; 2 LDS-window CSR (DPP); 3 LDS-densified
                                   * band on fp64 MFMA; 5 band-tile format (CSR densified once
                                   * into MFMA operand order, b in {16, 32}, |c - r| <= 64);
                                   * 6 segmented gather (power-law rows split / packed, b in
                                   * {16, 32}); 7 column panels (CSR rows in blocks of 256 / 512,
                                   * Q staged through LDS in 256-row panels of the columns a block
                                   * touches, b = 32; the default where every staged Q row is
                                   * read >= 4 times, i.e. bands wider than the band tiles' 64).
                                   * Each falls back 5 -> 3 -> 2 -> 1 (7 -> 1) when the matrix
                                   * does not fit the kernel's limits.  4 (dense panels) follows
                                   * from rbl_set_matrix_dense and is rejected here.           */
#define RBL_OPT_SPLIT_HALO    4   /* several ranks, band-tile SpMM: 1 (default) the kernel reads
                                   * the own rows from the block and the halo buffer holds only
                                   * the neighbours' rows; 0 the own block is copied into the
                                   * halo buffer every step (same results, bit for bit)         */
#define RBL_OPT_KEEP_CSR      5   /* 1 (default): the device CSR stays beside any SpMM format
                                   * built from it; 0: once the band tiles are built the CSR
                                   * (values, column ids, band positions, gather tables) is
                                   * released — 12 B per nonzero of HBM for the Krylov basis
                                   * (n = 5e7: 60 GB).  Then only b in {16, 32} can run and
                                   * rbl_get_matrix_csr fails.  Set before the matrix.          */
#define RBL_OPT_FUSE          6   /* pass fusions of the memory-bound b x b stages (b in {16, 32},
                                   * fp64 basis; default 7, all on):
                                   * bit 0: CholQR2 in 3 passes over the block instead of 4 (Q1
                                   *   recomputed, never stored) — bit for bit the same results;
                                   * bit 1: the next step's local-reorth Gram Q_i^T Q_{i+1} formed
                                   *   while the QR writes Q_{i+1} (used when that step runs no
                                   *   partial reorth), and Q_{i-1}^T Q_i by the last partial-
                                   *   reorth update — same results to rounding (1e-12);
                                   * bit 2: the local-reorth update Q_i -= Q_{i-1} C applied by
                                   *   the band-tile SpMM as it stages Q_i's rows (b = 32) — same
                                   *   results to rounding.  Works on several ranks: each rank
                                   *   corrects its first and last H rows (the rows its
                                   *   neighbours receive) before the halo exchange.  The
                                   *   several-rank form is tested with in-process ranks on one
                                   *   GPU; it has no run on several GPUs yet.               */

#define RBL_OPT_HALO_OVERLAP  7   /* several ranks, unbanded A (the segmented gather, whose halo is
                                   * most of Q_i): 1 (default) the halo exchange runs on a side
                                   * stream while the SpMM multiplies the own-column part of
                                   * each row, the halo-column part after it lands; 0 the same
                                   * two parts after the exchange (same results, bit for bit) */

#define RBL_OPT_RELABEL       8   /* 1: the next rbl_gen_matrix_rmat stores P A P^T for a seeded
                                   * permutation P (a Feistel bijection of the vertex ids): R-MAT's
                                   * hubs (its low ids) spread over the row range, so an
                                   * nnz-balanced row split gives every rank a like share of hub
                                   * and tail rows and of the halo it sends.  Eigenvalues are A's;
                                   * the device start block (omega NULL) draws row perm(v) from
                                   * v's id, so the run is the plain run permuted; rbl_row_ids gives
                                   * each local row's original id (a caller's omega and V rows are
                                   * in that order).  0 (default): A as drawn.                  */

#define RBL_OPT_HALO_PUSH     9   /* several ranks, unbanded A (the indexed halo of the segmented
                                   * gather), read when the matrix is set: each off-rank product
                                   * A[r,c] Q[c] is formed on the rank of the endpoint with the
                                   * larger (row degree, smaller id) — pulled Q[c] when that is c,
                                   * else computed by c's owner and its partial row pushed — so
                                   * the high-degree rows every rank references stay home and
                                   * only their partial rows move.  Needs A structurally
                                   * symmetric (checked from per-pair entry counts).  2 (default)
                                   * when its setup predicts fewer moved rows than pulling every
                                   * referenced row (< 0.85x); 1 always; 0 never.  Results differ
                                   * from the pull-all halo only in the order of each row's sum. */

typedef struct rbl_ctx rbl_ctx;

int rbl_abi_version(void);
/* How this copy of the library was built: RBL_BUILD_VARIANTS set when it was compiled with
 * -DRBL_VARIANTS (tools/build_variant.sh: the measured-and-rejected kernel variants and their
 * A/B switches, for diagnostics only; the product build leaves them out). */
#define RBL_BUILD_VARIANTS 1
int rbl_build_flags(void);

/* ---- context ------------------------------------------------------------------------
 * Replaces the implicit CUDA.jl device state of RBL_gpu.jl:1-6. */
int rbl_create(rbl_ctx** ctx, int device);
/* One rank of a row-partitioned multi-GPU job (one process per GPU).  `unique_id` is the
 * 128-byte RCCL id produced by rbl_get_unique_id() on rank 0 and broadcast by the host. */
int rbl_get_unique_id(uint8_t unique_id[128]);
/* Self-test of the RCCL transport on one device: a one-rank communicator (ncclCommInitRank)
 * runs the three collective shapes of a row-partitioned step — in-place all-reduce, host
 * all-gather, grouped send/recv — on device buffers and checks them.  msg (optional) gets a
 * one-line verdict.  RCCL refuses two ranks on one device, so a 1-GPU box can test no more. */
int rbl_comm_selftest(int device, char* msg, int msg_len);
int rbl_create_dist(rbl_ctx** ctx, int device, int nranks, int rank, const uint8_t unique_id[128]);
/* In-process rank group: `nranks` contexts in ONE process, each driven by its own host thread
 * (several may share a GPU).  Same multi-rank code path as rbl_create_dist with the RCCL
 * transport replaced by host-staged copies; used to exercise partitioning, halos and the
 * distributed Grams on a single-GPU machine.  The group is reference-counted: release it
 * with rbl_local_group_free whenever convenient (contexts keep it alive). */
typedef struct rbl_group rbl_group;
int rbl_local_group_create(rbl_group** group, int nranks);
int rbl_local_group_free(rbl_group* group);
int rbl_create_local(rbl_ctx** ctx, int device, rbl_group* group, int rank);
/* One rank of a process-per-rank job whose collectives go through a POSIX shared-memory
 * segment (host-staged, pinned) instead of RCCL: the production orchestration — one process
 * and one HIP context per rank, rendezvous, setup collectives, the side-stream halo exchange —
 * with ranks that may share one GPU (RCCL refuses that).  Every rank passes the same `path`
 * (e.g. "/dev/shm/rbl_<nonce>", unique per job); rank 0 creates it, the others wait for it,
 * and it is unlinked once all ranks have mapped it.  A rank that exits or stalls past
 * RBL_SHM_TIMEOUT_S seconds (default 120) makes its peers' calls fail with RBL_ERR_RCCL.
 * Transport name "shm" (rbl_comm_info). */
int rbl_create_shm(rbl_ctx** ctx, int device, int nranks, int rank, const char* path);
int rbl_free(rbl_ctx* ctx);
const char* rbl_last_error(const rbl_ctx* ctx);
/* Ranks as the transport itself counts them (RCCL: ncclCommCount; in-process group: its size;
 * one rank: 1, transport "none"), this context's rank, and the transport's name. */
int rbl_comm_info(rbl_ctx* ctx, int* nranks, int* rank, char* transport, int transport_len);
/* The RCCL library every RCCL-transport context calls: ROCm's own, opened by path
 * (/opt/rocm/lib/librccl.so.1, or $RBL_RCCL_LIB) with a private symbol scope, whatever else
 * the process loaded first (torch bundles another RCCL with the same soname).  version gets
 * ncclGetVersion's code (22707 = 2.27.7); path (optional) the file it was loaded from, or the
 * loader's error.  No GPU call: safe before any context exists. */
int rbl_rccl_version(int* version, char* path, int path_len);
int rbl_set_option(rbl_ctx* ctx, int option, int64_t value);
/* Free and total HBM of the context's device (hipMemGetInfo): what a caller checks before it
 * sizes a run (the reference sizes its buffer from CUDA.available_memory, RBL_gpu.jl:95-104). */
int rbl_device_memory(rbl_ctx* ctx, int64_t* free_bytes, int64_t* total_bytes);

/* ---- matrix --------------------------------------------------------------------------
 * Replaces `Ag = adapt(CuArray, A)` (RBL_gpu.jl:209).  The arrays are read as A's rows (CSR).
 * A is symmetric, so the CSC arrays of Julia's SparseMatrixCSC{Float64,Int64} are the CSR
 * arrays of A; `index_base` 1 accepts them unchanged.  For an unsymmetric A (benchmark.jl:58)
 * pass the CSC arrays of A^T — its CSR arrays — so the device computes A Q as cuSPARSE does
 * (julia/RBL_hip.jl and rbl.Context.set_matrix both do).  With nranks > 1 every rank passes the whole matrix and keeps the rows
 * [row_begin,row_end) of the nnz-balanced partition (rbl_plan_row_partition). */
int rbl_set_matrix_csc(rbl_ctx* ctx, int64_t n, int64_t nnz, const int64_t* colptr,
                       const int64_t* rowval, const double* nzval, int index_base);
/* Local CSR rows [row_begin,row_end) of an n x n symmetric matrix, global column ids. */
int rbl_set_matrix_csr_rows(rbl_ctx* ctx, int64_t n, int64_t row_begin, int64_t row_end,
                            const int64_t* rowptr, const int64_t* colind, const double* val,
                            int index_base);
/* Dense symmetric A (RBL_gpu(A::Matrix{Float64}, k, b), RBL_gpu.jl:205; images.jl's B^T B):
 * the local rows [row_begin,row_end) as a column-major slice with leading dimension lda
 * (one rank: the whole n x n matrix, lda >= n — Julia's Matrix pointer as-is).  A * Q then
 * runs as a panel GEMM on fp64 MFMA with Q gathered to all n rows on every rank.
 * rbl_spmm_kernel_for reports 4; rbl_get_matrix_csr fails (RBL_ERR_STATE). */
int rbl_set_matrix_dense(rbl_ctx* ctx, int64_t n, int64_t row_begin, int64_t row_end,
                         const double* A, int64_t lda);
/* Device-side generator of the seeded symmetric "hash-window" matrix:
 * entry (r,c), |r-c| <= halfwidth, r != c, exists iff hash(seed,min,max) < density, with a
 * uniform(-1,1) value from the same hash; diagonal = uniform(-1,1) plus plant[l] at row
 * l*floor(n/nplant) for l < nplant.  Each rank generates only its own rows. */
int rbl_gen_matrix_hashwindow(rbl_ctx* ctx, int64_t n, int64_t halfwidth, double density,
                              uint64_t seed, int nplant, const double* plant);
/* Device-side generator of the seeded symmetric R-MAT matrix (BASELINE
 * config 4): `edges` draws descend `scale` levels with quadrant probabilities (a, b, c,
 * 1-a-b-c); draws with an id >= n or a self loop are dropped, the rest enter as (r,c) and
 * (c,r), duplicates merged; off-diagonal values 2u-1 from the pair hash (as hash-window),
 * every diagonal entry present (hash value + planted spectrum, as hash-window).  Rows are
 * split over the ranks by nonzeros.  NumPy restatement: oracle/matgen.py rmat_csr. */
int rbl_gen_matrix_rmat(rbl_ctx* ctx, int64_t n, int scale, int64_t edges, double a, double b,
                        double c, uint64_t seed, int nplant, const double* plant);
/* Device-side generator of a circuit-like SPD matrix of SuiteSparse G3_circuit's shape
 * (BASELINE config 3; the real file is not shipped): a weighted graph Laplacian on a 5-point
 * stencil over rows of `width` nodes, each edge (lo,hi) kept iff hash(seed,lo,hi) < p_edge,
 * weight 0.5 + uniform[0,1) from the same hash; diagonal 0.01 + the kept weights (+ plant[l]
 * at node l*floor(n/nplant)); node i is scattered to row/column scatter(i), a seeded Feistel
 * bijection of [0,n), so the pattern has no band (the gather SpMM runs).  n = 1,585,478,
 * width 1259, p_edge 0.95873 give G3_circuit's 7.66 M nonzeros.  Rows split uniformly over
 * the ranks.  NumPy restatement: oracle/matgen.py circuit_like_csr. */
int rbl_gen_matrix_circuit(rbl_ctx* ctx, int64_t n, int64_t width, double p_edge, uint64_t seed,
                           int nplant, const double* plant);
int rbl_matrix_info(rbl_ctx* ctx, int64_t* n, int64_t* row_begin, int64_t* row_end,
                    int64_t* nnz_local);
/* Original (generator) id of each local row: r0 + i, or perm^-1(r0 + i) for a matrix generated
 * with RBL_OPT_RELABEL.  ids: n_local int64. */
int rbl_row_ids(rbl_ctx* ctx, int64_t* ids);
/* Download the local CSR (0-based) — test/inspection only. */
int rbl_get_matrix_csr(rbl_ctx* ctx, int64_t* rowptr, int32_t* colind, double* val);
/* Y = A X for a host n_local x b column-major block (the operator of RBL_gpu.jl:176,
 * `mul!(U, Ag, Qg_d)`), through the same SpMM kernels as rbl_step (multi-rank: with the
 * halo exchange).  Allocates its own device buffers. */
int rbl_apply(rbl_ctx* ctx, int b, const double* X, double* Y);
/* Which SpMM kernel rbl_step / rbl_apply use for block size b under the current option:
 * 1 = global-gather CSR, 2 = LDS-window CSR (DPP), 3 = LDS-densified band on fp64 MFMA,
 * 4 = dense panel GEMM (rbl_set_matrix_dense), 5 = band-tile format on fp64 MFMA,
 * 6 = segmented gather (unstructured patterns, b in {16, 32}). */
int rbl_spmm_kernel_for(rbl_ctx* ctx, int b);
/* The device format the matrix is held in: 0 = CSR only, 1 = band tiles (16 x (16 + 2H)
 * doubles), 2 = packed band tiles (RBL_BT_PACK=1), 3 = half band tiles (A symmetric bit for
 * bit: diagonal block + right strip, the left part transposed back in the kernel, same
 * results as 1; opt-in with RBL_BT_HALF=1), 4 = dense panels. */
int rbl_matrix_format(rbl_ctx* ctx);

/* ---- Krylov run -----------------------------------------------------------------------
 * rbl_start replaces RBL_gpu.jl:213-214 (`Qg_d = CUDA.randn(n,b); Qg_d = qr(Ag*Qg_d).Q`)
 * and the buffer planning of RBL_gpu.jl:95-104 (the whole basis lives in HBM).
 * `omega` is the local n_local x b column-major start block, or NULL for a device
 * counter-based N(0,1) draw from `seed`.  basis_bits: 64 (fp64 basis) or 32 (the mixed
 * mode of RBL_gpu.jl with FLOAT = Float32, any b: Krylov blocks and their partial /
 * local reorthogonalisation in fp32 on fp32 MFMA; A Q, the 3-term update, QR, A_i, B_i and
 * the Ritz projection in fp64 from the widened blocks). */
int rbl_start(rbl_ctx* ctx, int b, int max_blocks, int basis_bits, const double* omega,
              uint64_t seed);
/* One block Lanczos step i (1-based) — RBL_gpu.jl:149-161 for i == 1 and :163-184 for
 * i >= 2: partial reorth of Q_i, Q_{i-1} against Q_1..Q_{i-2} when bit 0 of `part_reorth`
 * is set (the reference sets it for even i; restarted.jl for i % 3 == 0), preceded by
 * their reorth against the locked vectors when bit 1 is set (restarted.jl:54-55; at i == 1
 * Q_1 alone, :41; fp64 basis only), local reorth, U = A Q_i - Q_{i-1} B_i^T,
 * A_i = Q_i^T U, U -= Q_i A_i, Q_{i+1} B_{i+1} = qr(U).  A_out/B_out: b x b column-major
 * host buffers receiving A_i and B_{i+1} (upper triangular) — the only per-step traffic. */
int rbl_step(rbl_ctx* ctx, int i, int part_reorth, double* A_out, double* B_out);
/* rbl_step without the per-step host round trip: the step is only enqueued; A_i, B_{i+1}
 * and its status are stashed in pinned memory and handed over by rbl_fetch.  Steps may be
 * enqueued back to back (the GPU never idles between them); the host fetches where it needs
 * the T band (the reference pushes every step, RBL_gpu.jl:185/193, but reads it only at the
 * convergence checks, :186-189).  A QR breakdown surfaces at the fetch. */
int rbl_step_async(rbl_ctx* ctx, int i, int part_reorth);
/* Wait for steps up to i1 - 1 and return those of [i0, i1) (i0 = the first unfetched step);
 * steps enqueued after i1 - 1 keep running (the host may enqueue ahead of a convergence check
 * and work on the T band meanwhile: with partial reorth at even steps, the steps after an even
 * i1 - 1 never touch blocks 1..i1-1):
 * A_out / B_out receive (i1-i0) consecutive b x b column-major blocks, status_out (may be
 * NULL) each step's status (RBL_OK, RBL_WARN_QR_SHIFTED, RBL_ERR_NUMERIC).  Returns
 * RBL_ERR_NUMERIC if any of them broke down, else RBL_OK.  rbl_step refuses to run while
 * asynchronous steps are unfetched. */
int rbl_fetch(rbl_ctx* ctx, int i0, int i1, double* A_out, double* B_out, int* status_out);
/* Ritz vectors — RBL_gpu.jl:106-132 / RBL.jl:61-71 in fp64:  V = [Q_1..Q_nblocks] S.
 * S: (nblocks*b) x k column-major (host); V_out: n_local x k column-major (host). */
int rbl_ritz(rbl_ctx* ctx, int nblocks, int k, const double* S, double* V_out);
/* Copy basis block j (1-based) to the host (n_local x b column-major) — tests only. */
int rbl_get_block(rbl_ctx* ctx, int j, double* Q_out);
int rbl_num_blocks(rbl_ctx* ctx);

/* ---- restarted variants (restarted.jl: RBL_gpu_restarted / RBL_restarted) ---------------
 * Locked Ritz vectors live on the device (Qlock_gpu); fp64 basis runs only.
 * rbl_restart: the next cycle starts from Q_1 = [Q_1..Q_nblocks] S (S: (nblocks*b) x b
 *   column-major), no QR — restarted.jl:131-132 `Qi = recover_eigvec(...)`; the locked set
 *   is kept, the block count resets to 1.
 * rbl_lock: append the nvec Ritz vectors [Q_1..Q_nblocks] S (S: (nblocks*b) x nvec) to the
 *   locked set — restarted.jl:121-126.  rbl_start empties the locked set.
 * rbl_reorth_last: the end-of-cycle reorth of Q_nblocks, Q_{nblocks-1} (flags as rbl_step's
 *   part_reorth) — restarted.jl:100-102. */
int rbl_restart(rbl_ctx* ctx, int nblocks, const double* S);
int rbl_lock(rbl_ctx* ctx, int nblocks, int nvec, const double* S);
int rbl_num_locked(rbl_ctx* ctx);
int rbl_get_locked(rbl_ctx* ctx, double* V_out);  /* n_local x num_locked column-major */
int rbl_reorth_last(rbl_ctx* ctx, int nblocks, int flags);

/* ---- timers --------------------------------------------------------------------------- */
int rbl_num_stages(void);
const char* rbl_stage_name(int stage);
int rbl_timers(rbl_ctx* ctx, double* ms, int nstages);
int rbl_reset_timers(rbl_ctx* ctx);
/* Stage times accumulate (ms, hipEvents on the context stream) while RBL_OPT_TIMERS is
 * set; names are the reference's TimerOutputs labels (RBL_gpu.jl:153-186: "AQ", "3-term",
 * "qr", "part reorth", "loc reorth", "Ritz vectors") plus "comm" (halo + all-reduce) and
 * "spill wait" (host spill: the stall on a block's copy-out).
 * rbl_synchronize waits for the context's stream and folds finished events into them. */
int rbl_synchronize(rbl_ctx* ctx);

/* Collectives this rank issued since the last reset (no reference equivalent: the reference is
 * single-GPU).  out[RBL_COMM_*] for the first nstats counters; reset != 0 zeroes them after the
 * read.  All-reduces are the b x b / (m b) x 2b Gram sums; exchanges the grouped halo
 * send/recv of Q rows before each SpMM (one rank: all zero). */
#define RBL_COMM_ALLREDUCE_CALLS 0
#define RBL_COMM_ALLREDUCE_BYTES 1
#define RBL_COMM_EXCHANGE_CALLS  2
#define RBL_COMM_SEND_BYTES      3
#define RBL_COMM_RECV_BYTES      4
#define RBL_COMM_NSTATS          5
/* the halo plan of the matrix held (set by rbl_set_matrix_* / the generators; reset keeps them):
 * RBL_COMM_HALO_PUSH 1 when the push/pull split runs (RBL_OPT_HALO_PUSH), and the Q rows per
 * SpMM summed over ranks that its setup predicted with the split (pulled + pushed) and with
 * the pull-all halo (0 on one rank or a banded A; the split's count also 0 when
 * RBL_OPT_HALO_PUSH is 0, which skips its evaluation) */
#define RBL_COMM_HALO_PUSH       5
#define RBL_COMM_PUSH_ROWS       6
#define RBL_COMM_PULL_ROWS       7
/* time in the collectives since the last reset, ns: host wall time inside the transport's calls
 * (all-reduces / halo exchanges; RCCL only enqueues, the shm and in-process stand-ins block),
 * and the hipEvent span each call holds its stream — the wait for the slowest peer included —
 * summed (recorded only while RBL_OPT_TIMERS is 1) */
#define RBL_COMM_ALLREDUCE_HOST_NS 8
#define RBL_COMM_EXCHANGE_HOST_NS  9
#define RBL_COMM_ALLREDUCE_DEV_NS  10
#define RBL_COMM_EXCHANGE_DEV_NS   11
int rbl_comm_stats(rbl_ctx* ctx, int64_t* out, int nstats, int reset);

/* All-gather of n int64 per rank from host memory: all[p*n + i] = rank p's mine[i] (one rank: a
 * copy).  A collective, ordered after the work already enqueued on the context (the host waits
 * for it).  The host loop uses it to take one decision for every rank — the convergence test
 * and the speculation depth of the next check (rbl.lanczos) — so that ranks whose host
 * eigensolves differ in the last bit still enqueue the same steps and collectives. */
int rbl_allgather_host(rbl_ctx* ctx, const int64_t* mine, int64_t* all, int n);

/* Which code path the block steps took, counted as the work is issued (since the last reset;
 * nstats entries, missing ones 0).  Stage timers cannot show this when ranks share a GPU (a
 * stage's events also span the other ranks' kernels); these counts are exact. */
#define RBL_PATH_SPMM            0  /* SpMM launches on a sparse A                              */
#define RBL_PATH_SPMM_LOC_FUSED  1  /* ... of which applied the local-reorth update to Q_i      */
#define RBL_PATH_LOC_SEPARATE    2  /* local-reorth updates run as their own pass              */
#define RBL_PATH_LOC_GRAM        3  /* local-reorth Grams not formed by the producing pass     */
#define RBL_PATH_LOCFIX_EDGES    4  /* rank-edge rows corrected before the halo exchange       */
#define RBL_PATH_LOCFIX_REST     5  /* range-edge rows corrected after a fused SpMM            */
#define RBL_PATH_SPMM_TWO_WAVE   6  /* SpMM launches served by the two-waves-per-SIMD kernel
                                       (variants build only; 0 in the product library)        */
#define RBL_PATH_RITZ_PIECES     7  /* rbl_ritz calls that formed V in row pieces on the side
                                       stream with the staged D2H behind them                  */
#define RBL_PATH_NSTATS          8
int rbl_path_stats(rbl_ctx* ctx, int64_t* out, int nstats, int reset);

/* ---- host-only planning (callable without a GPU) -------------------------------------- */
/* nnz-balanced contiguous row partition: bounds_out[0..nranks] (bounds_out[0]=0). */
int rbl_plan_row_partition(int64_t n, const int64_t* rowptr, int nranks, int64_t* bounds_out);
/* Column footprint of local rows: for each rank q, the contiguous global row range
 * [lo[q],hi[q]) of Q that the local rows reference within q's partition (lo==hi: none). */
int rbl_plan_halo(int64_t nrows_local, const int64_t* rowptr, const int64_t* colind,
                  int index_base, int nranks, const int64_t* bounds, int64_t* lo, int64_t* hi);
/* Hash-window generator on the host (same bits as the device generator): counts only
 * (rowptr_out, n_rows+1) when colind/val are NULL.  Rows [row_begin,row_end). */
int rbl_hashwindow_rows_host(int64_t n, int64_t halfwidth, double density, uint64_t seed,
                             int nplant, const double* plant, int64_t row_begin,
                             int64_t row_end, int64_t* rowptr_out, int64_t* colind_out,
                             double* val_out);

#ifdef __cplusplus
}
#endif
#endif /* RBL_HIP_H */
