#!/usr/bin/env python3
"""Round 6: is the slow-spectrum time-to-k's first-Ritz wait (DESIGN §5, 11-32 ms in bench.py's
order) CPU-quota throttling?  Replays bench.py's time-to-k order on one context (planted run and
time-to-k, matrix regenerated, slow-spectrum time-to-k x3) and prints, per slow run, its time,
Ritz + D2H, host eigensolve and the cgroup's throttled periods / microseconds during the run."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-randomized-block-lanczos_amd")]
import numpy as np  # noqa: E402
import rbl  # noqa: E402


def cpu_stat():
    out = {}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for line in f:
                k, v = line.split()
                out[k] = int(v)
    except OSError:
        pass
    return out


def vmstat():
    out = {}
    try:
        with open("/proc/vmstat") as f:
            for line in f:
                k_, v = line.split()
                if k_.startswith(("numa_", "pgmigrate", "thp_", "compact_stall", "allocstall")):
                    out[k_] = int(v)
    except OSError:
        pass
    return out


def delta(a, b, k):
    return b.get(k, 0) - a.get(k, 0)


try:
    quota = open("/sys/fs/cgroup/cpu.max").read().strip()
except OSError:
    quota = "n/a"
print(f"cpu.max {quota}; affinity {len(os.sched_getaffinity(0))} CPUs; "
      f"OMP_NUM_THREADS={os.environ.get('OMP_NUM_THREADS')}", flush=True)
n, b, k = 10_000_000, 32, 20
plant = np.array([100.0 * (2 * k + 1 - l) for l in range(1, 2 * k + 1)])
slow = np.array([12.0 + 0.25 * (2 * k + 1 - l) for l in range(1, 2 * k + 1)])
order = sys.argv[1] if len(sys.argv) > 1 else "bench"
# extra variants (argv[2]): "sleep" pauses 2 s before the first slow run; "prewarm" runs the host
# eigensolve on random bands of every check's size first (no GPU work)
extra = sys.argv[2] if len(sys.argv) > 2 else ""


try:
    print("numa_balancing", open("/proc/sys/kernel/numa_balancing").read().strip(), flush=True)
except OSError:
    print("numa_balancing n/a", flush=True)
if extra == "mpol":  # a task mempolicy without MPOL_F_MOF: NUMA balancing skips this task's VMAs
    import ctypes
    _libc = ctypes.CDLL("libc.so.6", use_errno=True)
    print("set_mempolicy(MPOL_LOCAL)", _libc.syscall(238, 4, None, 0), ctypes.get_errno(), flush=True)
if extra == "nohuge":  # numpy's madvise(MADV_HUGEPAGE) on arrays >= 4 MiB switched off
    from numpy._core import multiarray as _ma
    print("madvise_hugepage was", _ma._set_madvise_hugepage(False), flush=True)
if extra == "mallopt":  # heap policy: no mmap / munmap churn for arrays below 256 MiB
    import ctypes
    _libc = ctypes.CDLL("libc.so.6")
    print("mallopt", _libc.mallopt(-3, 256 << 20), _libc.mallopt(-1, 1 << 30), flush=True)


def prewarm_host(sizes=range(4, 29, 4)):
    from rbl.host import TBand, eig_topk
    rng = np.random.default_rng(0)
    for m in sizes:
        T = TBand(b, 38)
        for j in range(1, m + 1):
            a = rng.standard_normal((b, b))
            T.insert_A(a + a.T)
            T.insert_B(np.triu(rng.standard_normal((b, b))), j)
        eig_topk(T.view(), k)
with rbl.Context(0) as ctx:
    ctx.set_option(0, 1)
    if order == "bench":
        ctx.gen_hashwindow(n, 64, 0.7734, 20261015, plant)
        rbl.lanczos(ctx, k, b, check=False, ritz=False)
        D, V, info = rbl.lanczos(ctx, k, b, seed=3)
        print(f"planted: ritz+d2h={info.ritz_ms:.1f} eig={info.eig_ms:.1f}", flush=True)
        V = None
    ctx.gen_hashwindow(n, 64, 0.7734, 20261015, slow)
    ctx.start(b, 38, seed=3)
    ctx.step(1, False)
    ctx.synchronize()
    if extra == "sleep":
        time.sleep(2.0)
    elif extra == "tpc":
        from threadpoolctl import threadpool_limits
        with threadpool_limits(limits=1, user_api="blas"):
            pass
    elif extra == "eig896":
        prewarm_host([28])
    elif extra == "eig512":
        prewarm_host([16])
    elif extra == "alloc":
        for mb in range(1, 8):
            a = np.zeros((mb << 17,))
            a[:] = 1.0
            del a
    elif extra == "prewarm":
        t = time.perf_counter()
        prewarm_host()
        print(f"host prewarm {1e3 * (time.perf_counter() - t):.1f} ms", flush=True)
    for rep in range(3):
        ctx.synchronize()
        ctx.reset_timers()
        s0 = cpu_stat()
        v0 = vmstat()
        c0 = time.process_time()
        t = time.perf_counter()
        D, V, info = rbl.lanczos(ctx, k, b, seed=3)
        dt = time.perf_counter() - t
        c1 = time.process_time()
        s1 = cpu_stat()
        v1 = vmstat()
        print(f"{order}{('+' + extra) if extra else ''} slow rep {rep}: {dt * 1e3:7.1f} ms iters={info.iters} eig={info.eig_ms:.1f} "
              f"ritz+d2h={info.ritz_ms:.1f} cpu_s={c1 - c0:.2f} "
              f"throttled_periods={delta(s0, s1, 'nr_throttled')} "
              f"throttled_ms={delta(s0, s1, 'throttled_usec') / 1e3:.1f} "
              f"periods={delta(s0, s1, 'nr_periods')}", flush=True)
        print(f"   host: start={info.start_ms:.1f} enqueue={info.enqueue_ms:.1f} fetch_wait={info.fetch_ms:.1f} "
              f"eig={info.eig_ms:.1f} ritz={info.ritz_ms:.1f} spec={info.spec_steps}; stages "
              + " ".join(f"{k_}={v:.1f}" for k_, v in ctx.timers().items() if v), flush=True)
        print("   vmstat: " + " ".join(f"{k_}={v1[k_] - v0.get(k_, 0)}" for k_ in v1 if v1[k_] != v0.get(k_, 0)),
              flush=True)
        V = None
