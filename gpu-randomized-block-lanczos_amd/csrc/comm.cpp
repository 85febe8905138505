// comm.cpp — RCCL and in-process transports behind rbl::Comm (see comm.hpp).
#include "comm.hpp"

#include <dlfcn.h>
#include <rccl/rccl.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <mutex>

namespace rbl {

namespace {

// ---------------------------------------------------------------------------------------
// The RCCL this library calls is ROCm's own (/opt/rocm/lib/librccl.so.1, or $RBL_RCCL_LIB),
// opened here with RTLD_LOCAL | RTLD_DEEPBIND and called through the pointers below.  The
// library is not linked against RCCL: with a DT_NEEDED entry, a process that imported torch
// first had torch's bundled RCCL (same soname) serve every call, and one that did not had
// ROCm's — the copy depended on import order.  Opened by path, ROCm's copy is the one used in
// every process (a second copy beside torch's when torch is loaded; torch keeps its own); if
// that file does not load, RCCL is reported unavailable rather than looked up by soname.
struct RcclApi {
  bool ok = false;
  std::string path, error;
  int version = 0;
  decltype(&::ncclGetErrorString) GetErrorString = nullptr;
  decltype(&::ncclGetVersion) GetVersion = nullptr;
  decltype(&::ncclGetUniqueId) GetUniqueId = nullptr;
  decltype(&::ncclCommInitRank) CommInitRank = nullptr;
  decltype(&::ncclCommDestroy) CommDestroy = nullptr;
  decltype(&::ncclCommCount) CommCount = nullptr;
  decltype(&::ncclAllReduce) AllReduce = nullptr;
  decltype(&::ncclAllGather) AllGather = nullptr;
  decltype(&::ncclSend) Send = nullptr;
  decltype(&::ncclRecv) Recv = nullptr;
  decltype(&::ncclGroupStart) GroupStart = nullptr;
  decltype(&::ncclGroupEnd) GroupEnd = nullptr;
};

const RcclApi& rccl() {
  static RcclApi api;
  static std::once_flag once;
  std::call_once(once, [] {
    // by path only: a soname lookup ("librccl.so.1") in a process that imported torch first
    // would return torch's copy, the import-order dependence this loader exists to remove
    const char* env = std::getenv("RBL_RCCL_LIB");
    void* h = dlopen(env && *env ? env : "/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL | RTLD_DEEPBIND);
    if (!h) {
      api.error = dlerror();
      return;
    }
    bool all = true;
    auto sym = [&](auto& fp, const char* name) {
      fp = reinterpret_cast<std::remove_reference_t<decltype(fp)>>(dlsym(h, name));
      if (!fp) {
        all = false;
        api.error += std::string("; missing ") + name;
      }
    };
    sym(api.GetErrorString, "ncclGetErrorString");
    sym(api.GetVersion, "ncclGetVersion");
    sym(api.GetUniqueId, "ncclGetUniqueId");
    sym(api.CommInitRank, "ncclCommInitRank");
    sym(api.CommDestroy, "ncclCommDestroy");
    sym(api.CommCount, "ncclCommCount");
    sym(api.AllReduce, "ncclAllReduce");
    sym(api.AllGather, "ncclAllGather");
    sym(api.Send, "ncclSend");
    sym(api.Recv, "ncclRecv");
    sym(api.GroupStart, "ncclGroupStart");
    sym(api.GroupEnd, "ncclGroupEnd");
    if (!all) return;
    Dl_info di;
    if (dladdr(reinterpret_cast<void*>(api.AllReduce), &di) && di.dli_fname) api.path = di.dli_fname;
    if (api.GetVersion(&api.version) != ncclSuccess) api.version = 0;
    api.ok = true;
  });
  return api;
}

int hip_fail(hipError_t e, const char* what, std::string* err) {
  if (err) *err = std::string(what) + ": " + hipGetErrorString(e);
  return -2;  // RBL_ERR_HIP
}
int nccl_fail(ncclResult_t r, const char* what, std::string* err) {
  if (err) *err = std::string(what) + ": " + rccl().GetErrorString(r);
  return -4;  // RBL_ERR_RCCL
}

#define HIPX(expr)                                    \
  do {                                                \
    hipError_t _e = (expr);                           \
    if (_e != hipSuccess) return hip_fail(_e, #expr, err); \
  } while (0)
#define NCCLX(expr)                                      \
  do {                                                   \
    ncclResult_t _r = (expr);                            \
    if (_r != ncclSuccess) return nccl_fail(_r, #expr, err); \
  } while (0)

// ---------------------------------------------------------------------------------------
struct RcclComm final : Comm {
  ncclComm_t comm = nullptr;
  ~RcclComm() override {
    if (comm) rccl().CommDestroy(comm);
  }
  const char* name() const override { return "rccl"; }
  int count(int* n, std::string* err) override {
    NCCLX(rccl().CommCount(comm, n));
    return 0;
  }
  int allreduce_sum(double* dbuf, size_t count, hipStream_t st, std::string* err) override {
    NCCLX(rccl().AllReduce(dbuf, dbuf, count, ncclDouble, ncclSum, comm, st));
    return 0;
  }
  int allgather_host(const int64_t* mine, int64_t* all, size_t n, hipStream_t st,
                     std::string* err) override {
    int64_t *d_in = nullptr, *d_out = nullptr;
    HIPX(hipMalloc(&d_in, n * sizeof(int64_t)));
    HIPX(hipMalloc(&d_out, n * nranks * sizeof(int64_t)));
    HIPX(hipMemcpyAsync(d_in, mine, n * sizeof(int64_t), hipMemcpyHostToDevice, st));
    NCCLX(rccl().AllGather(d_in, d_out, n, ncclInt64, comm, st));
    HIPX(hipMemcpyAsync(all, d_out, n * nranks * sizeof(int64_t), hipMemcpyDeviceToHost, st));
    HIPX(hipStreamSynchronize(st));
    hipFree(d_in);
    hipFree(d_out);
    return 0;
  }
  int exchange(const std::vector<Xfer>& x, hipStream_t st, std::string* err) override {
    const RcclApi& api = rccl();
    NCCLX(api.GroupStart());
    for (int q = 0; q < nranks; ++q) {
      if (q == rank) continue;
      if (x[q].nsend) NCCLX(api.Send(x[q].send, x[q].nsend, ncclDouble, q, comm, st));
      if (x[q].nrecv) NCCLX(api.Recv(x[q].recv, x[q].nrecv, ncclDouble, q, comm, st));
    }
    NCCLX(api.GroupEnd());
    return 0;
  }
};

}  // namespace

int rccl_library(int* version, std::string* path, std::string* err) {
  const RcclApi& api = rccl();
  if (!api.ok) {
    if (err) *err = "RCCL not loaded: " + api.error;
    return -4;
  }
  if (version) *version = api.version;
  if (path) *path = api.path;
  return 0;
}

int rccl_unique_id(uint8_t unique_id[128]) {
  ncclUniqueId id;
  static_assert(sizeof(id) == 128, "ncclUniqueId size");
  if (!rccl().ok || rccl().GetUniqueId(&id) != ncclSuccess) return -4;
  memcpy(unique_id, &id, 128);
  return 0;
}

Comm* make_rccl_comm(int nranks, int rank, const uint8_t unique_id[128], std::string* err) {
  if (rccl_library(nullptr, nullptr, err)) return nullptr;
  auto* c = new RcclComm();
  c->nranks = nranks;
  c->rank = rank;
  ncclUniqueId id;
  memcpy(&id, unique_id, 128);
  const ncclResult_t r = rccl().CommInitRank(&c->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    nccl_fail(r, "ncclCommInitRank", err);
    c->comm = nullptr;
    delete c;
    return nullptr;
  }
  return c;
}

// ---------------------------------------------------------------------------------------
// In-process group.  Every collective is: publish (own slot) -> barrier -> consume (peers'
// slots) -> barrier.  A rank that never arrives (its thread failed) makes the others time
// out with an error instead of hanging.
struct LocalGroup {
  int nranks = 0;
  std::atomic<int> refs{1};
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  uint64_t generation = 0;
  bool broken = false;
  std::vector<std::vector<double>> red;       // allreduce contributions
  std::vector<std::vector<int64_t>> gath;     // allgather contributions
  std::vector<std::vector<Comm::Xfer>> xfer;  // exchange descriptors

  bool barrier() {
    std::unique_lock<std::mutex> lk(mu);
    if (broken) return false;
    const uint64_t gen = generation;
    if (++arrived == nranks) {
      arrived = 0;
      ++generation;
      cv.notify_all();
      return true;
    }
    const bool ok = cv.wait_for(lk, std::chrono::seconds(120),
                                [&] { return generation != gen || broken; });
    if (!ok || broken) {
      broken = true;
      cv.notify_all();
      return false;
    }
    return true;
  }
};

LocalGroup* local_group_create(int nranks) {
  auto* g = new LocalGroup();
  g->nranks = nranks;
  g->red.resize(nranks);
  g->gath.resize(nranks);
  g->xfer.resize(nranks);
  return g;
}

void local_group_release(LocalGroup* g) {
  if (g && g->refs.fetch_sub(1) == 1) delete g;
}

namespace {

struct LocalComm final : Comm {
  LocalGroup* g = nullptr;
  ~LocalComm() override { local_group_release(g); }
  const char* name() const override { return "local"; }

  int sync_barrier(std::string* err) {
    if (g->barrier()) return 0;
    if (err) *err = "local group barrier failed (a peer rank stopped or timed out)";
    return -4;
  }
  int allreduce_sum(double* dbuf, size_t count, hipStream_t st, std::string* err) override {
    auto& mine = g->red[rank];
    mine.resize(count);
    HIPX(hipMemcpyAsync(mine.data(), dbuf, count * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPX(hipStreamSynchronize(st));
    if (int s = sync_barrier(err)) return s;
    std::vector<double> sum(count, 0.0);
    for (int p = 0; p < nranks; ++p) {  // rank order: identical bits on every rank
      if (g->red[p].size() != count) {
        if (err) *err = "local allreduce: ranks disagree on the count";
        g->barrier();
        return -1;
      }
      for (size_t i = 0; i < count; ++i) sum[i] += g->red[p][i];
    }
    if (int s = sync_barrier(err)) return s;
    HIPX(hipMemcpyAsync(dbuf, sum.data(), count * sizeof(double), hipMemcpyHostToDevice, st));
    HIPX(hipStreamSynchronize(st));
    return 0;
  }
  int allgather_host(const int64_t* mine, int64_t* all, size_t n, hipStream_t st,
                     std::string* err) override {
    (void)st;
    g->gath[rank].assign(mine, mine + n);
    if (int s = sync_barrier(err)) return s;
    for (int p = 0; p < nranks; ++p) {
      if (g->gath[p].size() != n) {
        if (err) *err = "local allgather: ranks disagree on the count";
        g->barrier();
        return -1;
      }
      memcpy(all + (size_t)p * n, g->gath[p].data(), n * sizeof(int64_t));
    }
    return sync_barrier(err);
  }
  int exchange(const std::vector<Xfer>& x, hipStream_t st, std::string* err) override {
    HIPX(hipStreamSynchronize(st));  // what we send is complete before peers read it
    g->xfer[rank] = x;
    if (int s = sync_barrier(err)) return s;
    int rc = 0;
    for (int q = 0; q < nranks && rc == 0; ++q) {
      if (q == rank || x[q].nrecv == 0) continue;
      const Xfer& theirs = g->xfer[q][rank];
      if (theirs.nsend != x[q].nrecv) {
        if (err) *err = "local exchange: send/recv size mismatch";
        rc = -1;
        break;
      }
      const hipError_t e = hipMemcpyAsync(x[q].recv, theirs.send, x[q].nrecv * sizeof(double),
                                          hipMemcpyDefault, st);
      if (e != hipSuccess) rc = hip_fail(e, "hipMemcpyAsync(halo)", err);
    }
    if (rc == 0) {
      const hipError_t e = hipStreamSynchronize(st);
      if (e != hipSuccess) rc = hip_fail(e, "hipStreamSynchronize(halo)", err);
    }
    // second barrier: senders may not overwrite their rows until every reader is done
    const int s = sync_barrier(err);
    return rc ? rc : s;
  }
};

}  // namespace

Comm* make_local_comm(LocalGroup* g, int rank, std::string* err) {
  if (!g || rank < 0 || rank >= g->nranks) {
    if (err) *err = "make_local_comm: bad group or rank";
    return nullptr;
  }
  g->refs.fetch_add(1);
  auto* c = new LocalComm();
  c->g = g;
  c->nranks = g->nranks;
  c->rank = rank;
  return c;
}

}  // namespace rbl
