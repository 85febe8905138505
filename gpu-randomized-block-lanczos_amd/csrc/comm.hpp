// comm.hpp — the three collective shapes a row-partitioned block Lanczos step needs
// (SURVEY §8(e)): an in-place sum of small fp64 buffers (b x b / (m b) x 2b Gram
// coefficients), a host all-gather of a few int64 (slice bounds, halo tables) and a grouped
// point-to-point exchange of Q rows (the SpMM halo).
//
// Two transports:
//   * RcclComm  — production: one process per GPU, RCCL over xGMI (ncclAllReduce,
//                 ncclAllGather, grouped ncclSend/ncclRecv on the context's stream).
//   * LocalComm — every rank is a context in ONE process, each driven by its own host thread
//                 (several ranks may share one GPU).  It exists so the multi-rank code path —
//                 partitioning, halos, distributed Grams — runs on a single-GPU box, where RCCL
//                 refuses two ranks on one device.  Sums are formed on the host in rank order,
//                 so every rank gets bit-identical results (RCCL's guarantee too).
//   * ShmComm   — one PROCESS per rank, as in production, with the collectives staged through
//                 a POSIX shared-memory segment (host memory registered with HIP) instead of
//                 RCCL: the process-per-GPU orchestration (launcher, rendezvous, per-process
//                 HIP contexts, the setup collectives, the side-stream exchange) runs on a
//                 one-GPU box, where RCCL refuses two ranks on one device.  Same rank-order
//                 sums as LocalComm.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <string>
#include <vector>

namespace rbl {

struct Comm {
  int nranks = 1, rank = 0;
  virtual ~Comm() {}
  virtual const char* name() const = 0;
  // ranks the transport itself reports (RCCL: ncclCommCount), a cross-check of nranks
  virtual int count(int* n, std::string* err) {
    (void)err;
    *n = nranks;
    return 0;
  }
  // in-place sum over ranks of `count` doubles (device memory) ordered on `st`
  virtual int allreduce_sum(double* dbuf, size_t count, hipStream_t st, std::string* err) = 0;
  // blocking all-gather of `n` int64 per rank (host memory): all[p*n + i] = rank p's mine[i]
  virtual int allgather_host(const int64_t* mine, int64_t* all, size_t n, hipStream_t st,
                             std::string* err) = 0;
  // grouped exchange: for each peer q != rank, send send[q] (nsend[q] doubles) to q and receive
  // nrecv[q] doubles from q into recv[q] (device memory), ordered on `st`
  struct Xfer {
    const double* send = nullptr;
    size_t nsend = 0;
    double* recv = nullptr;
    size_t nrecv = 0;
  };
  virtual int exchange(const std::vector<Xfer>& x, hipStream_t st, std::string* err) = 0;
};

Comm* make_rccl_comm(int nranks, int rank, const uint8_t unique_id[128], std::string* err);
int rccl_unique_id(uint8_t unique_id[128]);
// the RCCL every RcclComm calls (ROCm's, opened by path: comm.cpp): ncclGetVersion's code
// (e.g. 22707 for 2.27.7) and the file it was loaded from
int rccl_library(int* version, std::string* path, std::string* err);

struct LocalGroup;
LocalGroup* local_group_create(int nranks);
void local_group_release(LocalGroup* g);  // drops one reference
Comm* make_local_comm(LocalGroup* g, int rank, std::string* err);

// `path`: a file name every rank passes (e.g. /dev/shm/rbl_<nonce>); rank 0 creates it, the
// others wait for it (bounded), and rank 0 unlinks it once every rank has mapped it.
Comm* make_shm_comm(int nranks, int rank, const char* path, std::string* err);

}  // namespace rbl
