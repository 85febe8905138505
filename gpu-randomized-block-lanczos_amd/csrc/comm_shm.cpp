// comm_shm.cpp — ShmComm: one process per rank, collectives staged through POSIX shared memory
// (see comm.hpp).
//
// Segment layout (one file, mapped MAP_SHARED by every rank):
//   [0, 4 KiB)      header: magic, sizes, barrier counter / generation, broken flag, rank pids
//   meta            nranks x nranks int64: row p = rank p's send sizes of the current exchange
//   data            nranks areas of `cap` bytes (RBL_SHM_CAP_MB, default 64 MiB), registered
//                   with HIP so the D2H / H2D copies are DMA from pinned pages
// Every collective is: copy own contribution into the own area -> barrier -> read the peers'
// areas -> barrier (the areas are then free for the next round).  Transfers larger than an area
// run in rounds.  A peer that exits (pid gone) or a wait past RBL_SHM_TIMEOUT_S (default 120 s)
// breaks the group: every rank then returns RBL_ERR_RCCL instead of hanging.
#include <fcntl.h>
#include <sched.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdlib>
#include <cstring>

#include "comm.hpp"

namespace rbl {

namespace {

constexpr uint64_t kShmMagic = 0x52424c5f53484d31ull;  // "RBL_SHM1"
constexpr size_t kHdrBytes = 4096;
constexpr int kShmMaxRanks = 64;

struct ShmHdr {
  uint64_t magic;
  int32_t nranks;
  int32_t pad;
  uint64_t cap, meta_off, data_off, total;
  std::atomic<uint32_t> attached;
  std::atomic<uint32_t> broken;
  std::atomic<uint32_t> count;
  std::atomic<uint32_t> gen;
  int32_t pid[kShmMaxRanks];
};
static_assert(sizeof(ShmHdr) <= kHdrBytes, "shm header");
static_assert(std::atomic<uint32_t>::is_always_lock_free, "cross-process atomics");

int hip_fail(hipError_t e, const char* what, std::string* err) {
  if (err) *err = std::string("shm transport: ") + what + ": " + hipGetErrorString(e);
  return -2;  // RBL_ERR_HIP
}
int shm_fail(const std::string& what, std::string* err) {
  if (err) *err = "shm transport: " + what;
  return -4;  // RBL_ERR_RCCL (transport failure)
}

#define HIPX(expr)                                         \
  do {                                                     \
    hipError_t _e = (expr);                                \
    if (_e != hipSuccess) return hip_fail(_e, #expr, err); \
  } while (0)

double env_seconds(const char* name, double dflt) {
  const char* v = std::getenv(name);
  if (!v) return dflt;
  const double s = std::atof(v);
  return s > 0 ? s : dflt;
}

struct ShmComm final : Comm {
  char* base = nullptr;
  size_t total = 0;
  ShmHdr* h = nullptr;
  size_t cap = 0;
  bool registered = false;
  double timeout_s = 120.0;

  ~ShmComm() override {
    if (registered) (void)hipHostUnregister(base + h->data_off);
    if (base) munmap(base, total);
  }
  const char* name() const override { return "shm"; }

  char* area(int p) const { return base + h->data_off + (size_t)p * cap; }
  int64_t* meta(int p) const { return reinterpret_cast<int64_t*>(base + h->meta_off) + (size_t)p * nranks; }

  // a peer whose process is gone breaks the group
  bool peer_gone() const {
    for (int p = 0; p < nranks; ++p) {
      if (p == rank || h->pid[p] <= 0) continue;
      if (kill(h->pid[p], 0) != 0 && errno == ESRCH) return true;
    }
    return false;
  }

  int barrier(std::string* err) {
    if (h->broken.load(std::memory_order_acquire)) return shm_fail("group broken (a peer failed)", err);
    const uint32_t g = h->gen.load(std::memory_order_acquire);
    if (h->count.fetch_add(1, std::memory_order_acq_rel) == (uint32_t)nranks - 1) {
      h->count.store(0, std::memory_order_relaxed);
      h->gen.store(g + 1, std::memory_order_release);
      return 0;
    }
    const auto t0 = std::chrono::steady_clock::now();
    auto tcheck = t0;
    for (uint64_t it = 0;; ++it) {
      if (h->gen.load(std::memory_order_acquire) != g) return 0;
      if (it < 2000) continue;  // the common case: peers a few microseconds behind
      if (it < 20000) {
        sched_yield();
        continue;
      }
      const timespec ts{0, 20000};
      nanosleep(&ts, nullptr);
      if ((it & 255) == 0) {
        if (h->broken.load(std::memory_order_acquire)) return shm_fail("group broken (a peer failed)", err);
        const auto now = std::chrono::steady_clock::now();
        if (std::chrono::duration<double>(now - tcheck).count() > 1.0) {
          tcheck = now;
          if (peer_gone()) {
            h->broken.store(1, std::memory_order_release);
            return shm_fail("a peer rank's process exited", err);
          }
        }
        if (std::chrono::duration<double>(now - t0).count() > timeout_s) {
          h->broken.store(1, std::memory_order_release);
          return shm_fail("barrier timed out (RBL_SHM_TIMEOUT_S)", err);
        }
      }
    }
  }

  int allreduce_sum(double* dbuf, size_t count, hipStream_t st, std::string* err) override {
    const size_t chunk = cap / sizeof(double);
    std::vector<double> sum;
    for (size_t o = 0; o < count; o += chunk) {
      const size_t c = std::min(chunk, count - o);
      double* mine = reinterpret_cast<double*>(area(rank));
      HIPX(hipMemcpyAsync(mine, dbuf + o, c * sizeof(double), hipMemcpyDeviceToHost, st));
      HIPX(hipStreamSynchronize(st));
      if (int s = barrier(err)) return s;
      sum.assign(c, 0.0);
      for (int p = 0; p < nranks; ++p) {  // rank order: the same bits on every rank
        const double* a = reinterpret_cast<const double*>(area(p));
        for (size_t i = 0; i < c; ++i) sum[i] += a[i];
      }
      if (int s = barrier(err)) return s;
      HIPX(hipMemcpyAsync(dbuf + o, sum.data(), c * sizeof(double), hipMemcpyHostToDevice, st));
      HIPX(hipStreamSynchronize(st));
    }
    return 0;
  }

  int allgather_host(const int64_t* mine, int64_t* all, size_t n, hipStream_t st,
                     std::string* err) override {
    (void)st;
    const size_t chunk = cap / sizeof(int64_t);
    for (size_t o = 0; o < n || (o == 0 && n == 0); o += chunk) {
      const size_t c = std::min(chunk, n - o);
      memcpy(area(rank), mine + o, c * sizeof(int64_t));
      if (int s = barrier(err)) return s;
      for (int p = 0; p < nranks; ++p) memcpy(all + (size_t)p * n + o, area(p), c * sizeof(int64_t));
      if (int s = barrier(err)) return s;
      if (n == 0) break;
    }
    return 0;
  }

  int exchange(const std::vector<Xfer>& x, hipStream_t st, std::string* err) override {
    const int P = nranks, me = rank;
    HIPX(hipStreamSynchronize(st));  // what we send is complete
    int64_t* mrow = meta(me);
    for (int q = 0; q < P; ++q) mrow[q] = q == me ? 0 : (int64_t)x[q].nsend;
    if (int s = barrier(err)) return s;
    std::vector<int64_t> ns((size_t)P * P), off((size_t)P * P);
    for (int p = 0; p < P; ++p) memcpy(&ns[(size_t)p * P], meta(p), P * sizeof(int64_t));
    bool mismatch = false;
    size_t rounds = 0;
    const size_t capd = cap / sizeof(double);
    for (int p = 0; p < P; ++p) {
      int64_t o = 0;
      for (int q = 0; q < P; ++q) {
        off[(size_t)p * P + q] = o;
        o += ns[(size_t)p * P + q];
      }
      rounds = std::max(rounds, ((size_t)o + capd - 1) / capd);
    }
    for (int q = 0; q < P; ++q)
      if (q != me && ns[(size_t)q * P + me] != (int64_t)x[q].nrecv) mismatch = true;
    if (rounds == 0) {  // nothing moves: one barrier so the size table may be rewritten
      if (int s = barrier(err)) return s;
    }
    for (size_t r = 0; r < rounds; ++r) {
      const int64_t lo = (int64_t)(r * capd), hi = lo + (int64_t)capd;
      // pack: my sends that fall into [lo, hi) of my send stream
      for (int q = 0; q < P; ++q) {
        const int64_t s0 = off[(size_t)me * P + q], s1 = s0 + ns[(size_t)me * P + q];
        const int64_t a = std::max(s0, lo), e = std::min(s1, hi);
        if (e <= a) continue;
        HIPX(hipMemcpyAsync(area(me) + (a - lo) * sizeof(double), x[q].send + (a - s0),
                            (e - a) * sizeof(double), hipMemcpyDefault, st));
      }
      HIPX(hipStreamSynchronize(st));
      if (int s = barrier(err)) return s;
      // unpack: what each peer sends me within its [lo, hi)
      if (!mismatch) {
        for (int q = 0; q < P; ++q) {
          if (q == me) continue;
          const int64_t s0 = off[(size_t)q * P + me], s1 = s0 + ns[(size_t)q * P + me];
          const int64_t a = std::max(s0, lo), e = std::min(s1, hi);
          if (e <= a) continue;
          HIPX(hipMemcpyAsync(x[q].recv + (a - s0), area(q) + (a - lo) * sizeof(double),
                              (e - a) * sizeof(double), hipMemcpyDefault, st));
        }
        HIPX(hipStreamSynchronize(st));
      }
      if (int s = barrier(err)) return s;
    }
    if (mismatch) return shm_fail("exchange: a peer's send size differs from my receive size", err);
    return 0;
  }
};

}  // namespace

Comm* make_shm_comm(int nranks, int rank, const char* path, std::string* err) {
  if (!path || !*path || nranks < 1 || nranks > kShmMaxRanks || rank < 0 || rank >= nranks) {
    if (err) *err = "shm transport: bad path / nranks / rank";
    return nullptr;
  }
  const char* capv = std::getenv("RBL_SHM_CAP_MB");
  size_t cap = (size_t)(capv && std::atoll(capv) > 0 ? std::atoll(capv) : 64) << 20;
  cap = (cap + 4095) & ~size_t(4095);
  const size_t meta_off = kHdrBytes;
  const size_t data_off = (meta_off + (size_t)nranks * nranks * sizeof(int64_t) + 4095) & ~size_t(4095);
  const size_t total = data_off + (size_t)nranks * cap;
  const double timeout_s = env_seconds("RBL_SHM_TIMEOUT_S", 120.0);
  auto* c = new ShmComm();
  c->nranks = nranks;
  c->rank = rank;
  c->cap = cap;
  c->timeout_s = timeout_s;
  auto bail = [&](const std::string& m) -> Comm* {
    if (err) *err = "shm transport: " + m;
    delete c;
    return nullptr;
  };
  int fd = -1;
  if (rank == 0) {
    fd = open(path, O_RDWR | O_CREAT | O_EXCL, 0600);
    if (fd < 0) return bail(std::string("create ") + path + ": " + strerror(errno));
    // reserve the pages now: a full /dev/shm fails here instead of faulting (SIGBUS) later
    const int fe = posix_fallocate(fd, 0, (off_t)total);
    if (fe != 0) {
      close(fd);
      unlink(path);
      return bail(std::string("posix_fallocate: ") + strerror(fe));
    }
    void* m = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    if (m == MAP_FAILED) {
      close(fd);
      unlink(path);
      return bail(std::string("mmap: ") + strerror(errno));
    }
    c->base = static_cast<char*>(m);
    c->total = total;
    c->h = reinterpret_cast<ShmHdr*>(c->base);
    c->h->nranks = nranks;
    c->h->cap = cap;
    c->h->meta_off = meta_off;
    c->h->data_off = data_off;
    c->h->total = total;
    __atomic_store_n(&c->h->magic, kShmMagic, __ATOMIC_RELEASE);
  } else {
    const auto t0 = std::chrono::steady_clock::now();
    for (;;) {
      fd = open(path, O_RDWR);
      if (fd >= 0) {
        struct stat sb;
        if (fstat(fd, &sb) == 0 && (size_t)sb.st_size >= total) {
          void* m = mmap(nullptr, total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
          if (m == MAP_FAILED) {
            close(fd);
            return bail(std::string("mmap: ") + strerror(errno));
          }
          auto* hh = reinterpret_cast<ShmHdr*>(m);
          if (__atomic_load_n(&hh->magic, __ATOMIC_ACQUIRE) == kShmMagic) {
            if (hh->nranks != nranks || hh->cap != cap || hh->total != total) {
              munmap(m, total);
              close(fd);
              return bail("the segment's geometry differs (nranks / RBL_SHM_CAP_MB disagree)");
            }
            c->base = static_cast<char*>(m);
            c->total = total;
            c->h = hh;
            break;
          }
          munmap(m, total);
        }
        close(fd);
        fd = -1;
      }
      if (std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > timeout_s)
        return bail(std::string("rank 0 never created ") + path);
      const timespec ts{0, 1000000};
      nanosleep(&ts, nullptr);
    }
  }
  close(fd);
  c->h->pid[rank] = (int32_t)getpid();
  c->h->attached.fetch_add(1, std::memory_order_acq_rel);
  // pinned data areas: the stream copies are DMA (pageable memory would bounce through the
  // runtime's staging buffer); without it the transport still works, only slower
  c->registered = hipHostRegister(c->base + data_off, (size_t)nranks * cap, hipHostRegisterDefault) == hipSuccess;
  if (!c->registered) (void)hipGetLastError();
  std::string berr;
  if (c->barrier(&berr) != 0) {
    if (rank == 0) unlink(path);
    return bail(berr.substr(std::min<size_t>(berr.size(), 15)));
  }
  if (rank == 0) unlink(path);  // every rank has it mapped: no file outlives the group
  return c;
}

}  // namespace rbl
