#!/usr/bin/env python3
"""bench.py — RBL iterations/sec on the north-star workload (BASELINE.json `metric`).

Workload: seeded symmetric hash-window matrix, n = 1e7, ~100 nnz/row
(half-width 64, density 0.7734), planted top spectrum, b = 32, k = 20, generated on the
device (no host copy).  One bench "step" = one fixed-length RBL run: rbl_start (A*Omega +
QR) and the m_max = ceil(1200/b) = 38 block iterations of RBL_gpu.jl:162 with convergence
checks off (partial-reorth cost grows with i, so the step range is fixed).
value = block iterations per second of the whole job.  Time-to-k=20 (convergence on, from
start through Ritz vectors) is reported beside it.

Multi-GPU: one process per GPU (torch.distributed.run); rows are partitioned over ranks
(strong scaling: n fixed), SpMM halos and Gram all-reduces go over RCCL inside
librbl_hip.so; torch.distributed (gloo) only carries the RCCL id, barriers and the max-time.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "gpu-randomized-block-lanczos_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402

BASELINE_METRIC = ("RBL iters/sec + time-to-k=20 eigenpairs, n=1e7 nnz/row=100 b=32; "
                   "1/2/4/8 GPU")   # BASELINE.json "metric", quoted on C4a at N GPUs
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec (MI355X_MICROARCH.md)
FP64_MFMA_PEAK_TF = 78.6     # MI355X dense fp64 matrix spec
FP32_MFMA_PEAK_TF = 157.3    # MI355X dense fp32 matrix spec (v_mfma_f32_16x16x4_f32)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="GPUs (one process each).  Under torch.distributed.run it must equal "
                         "WORLD_SIZE; without it, N > 1 re-launches this script under "
                         "torch.distributed.run with N processes (before any GPU call)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--n", type=int, default=10_000_000)
    ap.add_argument("--b", type=int, default=32)
    ap.add_argument("--k", type=int, default=20)
    ap.add_argument("--halfwidth", type=int, default=64)
    ap.add_argument("--density", type=float, default=0.7734)
    ap.add_argument("--seed", type=int, default=20261015)
    ap.add_argument("--kryl", type=int, default=1200)
    ap.add_argument("--cpu-sample-n", type=int, default=100_000,
                    help="rows of the CPU baseline's sample (same generator, same block steps)")
    ap.add_argument("--no-cpu-one-thread", action="store_true",
                    help="skip the CPU baseline's second timing at 1 BLAS thread (benchmark.jl:49 "
                         "sets BLAS.set_num_threads(1); on by default)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-check-n", type=int, default=1_000_000,
                    help="n of the CPU baseline's fixed-step cross-check (0 skips it): the first "
                         "--cpu-check-steps block steps timed at the sample's n and at this n")
    ap.add_argument("--cpu-check-steps", type=int, default=8)
    ap.add_argument("--cpu-fixed-n", type=int, default=-1,
                    help="also time the oracle's first --cpu-check-steps block steps at this n (SURVEY "
                         "§8(d)'s fixed-step form at the config's own n: the 1e9-nnz CSR built in "
                         "row chunks, ~45 GB of host memory, ~3-4 minutes at n = 1e7 on 16 threads); "
                         "-1 (default): the run's own n on the hash-window matrix; 0: off")
    ap.add_argument("--no-ttk", action="store_true")
    ap.add_argument("--no-ttk-slow", action="store_true",
                    help="skip the second time-to-k on a slowly decaying planted spectrum "
                         "(12 + 0.25 (2k+1-l), l = 1..2k: its top eigenvalues sit just above the "
                         "bulk, as the reference's slow_dec suite, so convergence takes ~24 steps)")
    ap.add_argument("--speculate", choices=["auto", "off"], default="auto",
                    help="time-to-k runs: steps enqueued ahead of a convergence check while the "
                         "host solves the T band (rbl.lanczos speculate; 'off': the strict order)")
    ap.add_argument("--traffic-json", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--spmm-kernel", type=int, default=0)
    ap.add_argument("--matrix", default="hashwindow", choices=("hashwindow", "rmat", "circuit"),
                    help="rmat: BASELINE config 4's power-law pattern (SURVEY §8(d) C4b); "
                         "circuit: BASELINE config 3's shape (G3_circuit-like SPD Laplacian, "
                         "scattered; use --n 1585478 --b 16)")
    ap.add_argument("--wide-steps", type=int, default=2,
                    help="timed runs of the wide-band sub-record (0: skip)")
    ap.add_argument("--wide-halfwidth", type=int, default=1024,
                    help="half-width of the wide-band sub-record's hash-window matrix")
    ap.add_argument("--c3-steps", type=int, default=6,
                    help="timed runs of the C3 circuit sub-record that follows a hash-window run "
                         "(n = 1,585,478, b = 16, k = 20: BASELINE config 3's shape; 0 skips it)")
    ap.add_argument("--c5-steps", type=int, default=2,
                    help="timed runs of the C5 sub-record (BASELINE config 5: n = 5e7, ~100 nnz/row, "
                         "fp32 Krylov basis, b = 32) that follows a hash-window run on two or more "
                         "ranks, where the basis fits in HBM without spilling; 0 skips it")
    ap.add_argument("--c5-n", type=int, default=50_000_000)
    ap.add_argument("--c5-min-ranks", type=int, default=2,
                    help="fewest ranks the C5 sub-record runs on (one GPU would spill the 243 GB "
                         "fp32 basis to host memory: DESIGN §2)")
    ap.add_argument("--rmat-scale", type=int, default=24)
    ap.add_argument("--rmat-steps", type=int, default=3,
                    help="timed runs of the C4b R-MAT sub-record that follows a hash-window "
                         "run (BASELINE config 4 in the same job; 0 skips it)")
    ap.add_argument("--rmat-warmup", type=int, default=1)
    ap.add_argument("--halo-push", type=int, default=2, choices=(0, 1, 2),
                    help="RBL_OPT_HALO_PUSH for the unbanded sub-records on several ranks: the "
                         "push/pull split of the indexed halo (2: when its setup predicts fewer "
                         "moved rows)")
    ap.add_argument("--rmat-relabel", default="1", choices=("auto", "0", "1"),
                    help="RBL_OPT_RELABEL for the R-MAT matrix: store P A P^T for a seeded vertex "
                         "permutation (Graph500's generator scrambles its vertex ids the same way), "
                         "so R-MAT's hubs (its low ids) spread over the row range: the nnz-balanced "
                         "split then balances the halo each rank sends (P = 8: busiest sender 1.06x "
                         "the mean instead of 2.1x), and on one GPU the gather SpMM runs 34.3 "
                         "instead of 37.5 ms per launch (profiles/r04_bench_rmat_relabel*.json); "
                         "auto = on for several ranks only")
    ap.add_argument("--rmat-as-drawn-steps", type=int, default=1,
                    help="timed runs of the R-MAT matrix as drawn (no relabel) after the relabelled "
                         "sub-record, so the line stays comparable with rounds before the relabel "
                         "(0 skips it)")
    ap.add_argument("--rmat-edges", type=int, default=0,
                    help="R-MAT draws (0: 0.66 n x 100: ~1e9 nonzeros at n = 1e7 after merging)")
    ap.add_argument("--device-blocks", type=int, default=0,
                    help="Krylov blocks kept in HBM (RBL_OPT_DEVICE_BLOCKS; older blocks spill to "
                         "pinned host memory, the reference's hybrid buffer); 0 = all")
    ap.add_argument("--keep-csr", type=int, default=1, choices=(0, 1),
                    help="0: release the device CSR once the band tiles are built "
                         "(RBL_OPT_KEEP_CSR; frees 12 B per nonzero for the basis at n = 5e7)")
    ap.add_argument("--fuse", type=int, default=7, choices=tuple(range(8)),
                    help="RBL_OPT_FUSE: bit 0 the 3-pass CholQR2, bit 1 the local-reorth Gram formed "
                         "by the producing QR / partial-reorth update, bit 2 the local-reorth "
                         "update applied by the band-tile SpMM (A/B switch)")
    ap.add_argument("--transport", default="rccl", choices=("rccl", "shm"),
                    help="collectives between the rank processes: rccl (production, one GPU per "
                         "rank) or shm (rbl_create_shm: host-staged through POSIX shared memory; "
                         "ranks may share a GPU, so N ranks run on a one-GPU box — a rehearsal "
                         "of the multi-process path, not a scaling measurement)")
    ap.add_argument("--basis-bits", type=int, default=64, choices=(64, 32),
                    help="32: the mixed mode (fp32 Krylov basis + reorth on fp32 MFMA, fp64 A*Q / "
                         "3-term / QR) of BASELINE config 5, on this workload")
    argv = sys.argv[1:]
    if argv == ["--argv-env"]:  # re-launched by launch_ranks: the arguments travel in the env
        argv = json.loads(os.environ["RBL_BENCH_ARGV"])
    return ap.parse_args(argv)


def streamed_bytes(kid, nloc, nnz_loc, b, halfwidth, m_max, fmt=1):
    """Bytes the chosen SpMM kernel itself reads and writes per launch (step launches carry the
    Q_{i-1} epilogue), beside SURVEY's CSR-based algorithmic bytes: the band-tile kernel (5)
    streams 16 x (16 + 2H) dense doubles per 16-row tile instead of 12 B per nonzero; the
    LDS-band kernel (3) 8 B value + 2 B position per nonzero plus the row pointers.  Packed
    band tiles (RBL_BT_PACK=1; dense by default) stream the nonzeros and a header of 24
    (H = 32) or 42 (H = 64) 8-B words per tile; half band tiles (format 3, opt-in with
    RBL_BT_HALF=1 for a symmetric A; measured no faster) the diagonal block and the right strip, 16 x (16 + H) doubles per tile (the
    left part is the previous tiles' strips again, read back through L2)."""
    vec = (m_max * 3 + 2) / (m_max + 1) * nloc * b * 8
    if kid == 5:
        H = 32 if halfwidth <= 32 else 64
        tiles = -(-nloc // 16)
        if fmt == 2:
            return nnz_loc * 8 + tiles * 8 * (24 if H == 32 else 42) + vec
        if fmt == 3:
            return tiles * 16 * (16 + H) * 8 + vec
        return tiles * 16 * (16 + 2 * H) * 8 + vec
    if kid == 3:
        return nnz_loc * 10 + (nloc + 1) * 8 + vec
    return nnz_loc * 12 + (nloc + 1) * 8 + vec


def gpu_count_sysfs():
    """GPUs this process may use, without touching the HIP runtime: the visible-devices list
    if one is set, else the KFD topology nodes with a GPU (gfx_target_version != 0).  None when
    neither is readable (then the ranks find out themselves)."""
    for var in ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is not None:
            return len([x for x in v.split(",") if x.strip() != ""])
    base = "/sys/class/kfd/kfd/topology/nodes"
    try:
        nodes = os.listdir(base)
    except OSError:
        return None
    count = 0
    for nd in nodes:
        try:
            with open(os.path.join(base, nd, "properties")) as f:
                for line in f:
                    key, _, val = line.partition(" ")
                    if key == "gfx_target_version" and int(val) != 0:
                        count += 1
                        break
        except (OSError, ValueError):
            continue
    return count


def launch_ranks(args) -> None:
    """`--gpus N` outside torch.distributed.run: check the GPUs exist (KFD sysfs, no HIP call:
    this launcher process never initialises the GPU runtime), then run this script under
    torch.distributed.run with N processes and exit with its status."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if args.gpus is not None and args.gpus != int(env_world):
            sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world}")
        return
    if args.gpus is None or args.gpus <= 1:
        return
    import subprocess
    import socket
    have = gpu_count_sysfs()
    # the shm transport may put several ranks on one GPU (RCCL refuses that, unless each rank
    # declares its own host: the one-GPU rehearsal of the RCCL path, RBL_RCCL_HOST_PER_RANK=1)
    if (have is not None and have < args.gpus and args.transport != "shm"
            and not rccl_host_per_rank()):
        sys.exit(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, this node has {have}")
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    # the bench's own arguments go through the environment: torch.distributed.run's parser
    # would take some of them (`--n` is an ambiguous abbreviation of its options)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__), "--argv-env"]
    env = dict(os.environ, RBL_BENCH_ARGV=json.dumps(sys.argv[1:]))
    if have and have < args.gpus:  # (the box exports HIP's default 4: lowered, never raised)
        cur = int(env.get("GPU_MAX_HW_QUEUES") or 4)
        env["GPU_MAX_HW_QUEUES"] = str(min(cur, shared_gpu_queues(-(-args.gpus // have))))
    sys.exit(subprocess.run(cmd, env=env).returncode)


# Processes sharing one GPU in the rehearsals (measured, DESIGN.md §6, profiles/r06_p8_*): up to
# 6 run at the P = 4 rate per collective with HIP's default 4 hardware queues each; 7 and 8
# processes time-slice (every collective then waits ~10-45 ms) with 4 or 3 queues each, and run
# at the P = 4 rate again with 1 (the streams of a process then share its one queue).
SHARED_GPU_FULL_QUEUES_UP_TO = 6


def shared_gpu_queues(ranks_per_gpu: int) -> int:
    """GPU_MAX_HW_QUEUES for ranks that share a GPU (the rehearsal of an N-GPU job on fewer
    GPUs; never set for one rank per GPU)."""
    return 4 if ranks_per_gpu <= SHARED_GPU_FULL_QUEUES_UP_TO else 1


def rccl_host_per_rank() -> bool:
    """RBL_RCCL_HOST_PER_RANK=1 (a rehearsal on a box with fewer GPUs than ranks, not a
    measurement): every rank declares its own RCCL host id, so RCCL connects ranks that share a
    GPU through its network transport on the loopback interface instead of refusing them; the
    ranks go round-robin over the GPUs there are."""
    return os.environ.get("RBL_RCCL_HOST_PER_RANK", "0") == "1"


def rmat_relabel(args, world: int) -> int:
    """RBL_OPT_RELABEL for the R-MAT matrix (--rmat-relabel; auto: on for several ranks)."""
    return int(world > 1) if args.rmat_relabel == "auto" else int(args.rmat_relabel)


def workload_name(args) -> str:
    """BASELINE.json config this run measures, by its shape."""
    if args.matrix == "circuit":
        return ("C3-shaped circuit SpMM-Lanczos" if (args.n, args.b) == (1_585_478, 16)
                else "circuit-like SpMM-Lanczos")
    if args.matrix == "rmat":
        return "C4b R-MAT SpMM-Lanczos" if args.n == 10_000_000 and args.b == 32 else "R-MAT SpMM-Lanczos"
    if args.basis_bits == 32 and args.n == 50_000_000 and args.b == 32:
        return "C5 hash-window SpMM-Lanczos, mixed precision (fp32 basis)"
    tag = {(10_000_000, 32): "C4a", (1_000_000, 16): "C2"}.get((args.n, args.b))
    name = f"{tag} hash-window SpMM-Lanczos" if tag else "hash-window SpMM-Lanczos"
    if args.basis_bits == 32:
        name += ", mixed precision (fp32 basis, config 5 mode)"
    return name


def metric_name(args, nnz: int) -> str:
    """BASELINE.json's metric string for its own config; the same form for any other shape."""
    if (args.matrix == "hashwindow" and args.n == 10_000_000 and args.b == 32 and args.k == 20
            and args.basis_bits == 64):
        return BASELINE_METRIC
    return (f"RBL iters/sec + time-to-k={args.k} eigenpairs, n={args.n:.0e} "
            f"nnz/row={nnz / args.n:.0f} b={args.b}" + (" fp32 basis" if args.basis_bits == 32 else "")
            + f" ({args.matrix})")


T_START = time.perf_counter()


def progress(msg: str) -> None:
    """One line on stderr from rank 0 per phase and per fixed-length run: the JSON line is the
    only stdout, and a long multi-rank job must not look silent (gpurun ends a run that writes
    nothing for 3 minutes)."""
    if os.environ.get("RANK", "0") == "0":
        print(f"[bench {time.perf_counter() - T_START:7.1f} s] {msg}", file=sys.stderr, flush=True)


def host_threads() -> dict:
    """This process's threads by name (/proc/self/task/*/comm): RCCL's proxy / socket threads,
    HIP's, BLAS workers, the Python main thread."""
    names = {}
    try:
        for t in os.listdir("/proc/self/task"):
            try:
                with open(f"/proc/self/task/{t}/comm") as f:
                    nm = f.read().strip()
            except OSError:
                continue
            names[nm] = names.get(nm, 0) + 1
    except OSError:
        pass
    return dict(sorted(names.items(), key=lambda kv: -kv[1]))


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def cgroup_cpu() -> dict:
    """The CPU quota of this process's cgroup (v2 cpu.max or v1 cfs quota / period) and its
    throttling counters: a rehearsal whose ranks together want more CPU than the quota is
    throttled (every thread of the cgroup stopped until the next period) however many CPUs the
    affinity mask lists."""
    out = {}
    mx = _read("/sys/fs/cgroup/cpu.max")
    if mx:
        q, _, per = mx.partition(" ")
        out["quota_cpus"] = None if q == "max" else round(int(q) / int(per or 100000), 2)
        st = _read("/sys/fs/cgroup/cpu.stat") or ""
    else:
        q, per = _read("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"), _read("/sys/fs/cgroup/cpu/cpu.cfs_period_us")
        if q and per:
            out["quota_cpus"] = None if int(q) < 0 else round(int(q) / int(per), 2)
        st = _read("/sys/fs/cgroup/cpu/cpu.stat") or ""
    for line in st.splitlines():
        k, _, v = line.partition(" ")
        if k in ("nr_periods", "nr_throttled", "throttled_usec", "throttled_time", "usage_usec"):
            out[k] = int(v)
    return out


def gpu_processes() -> dict:
    """GPU processes the KFD driver knows on this node (/sys/class/kfd/kfd/proc: one entry per
    process with a GPU context), this process's queues there, and the amdgpu scheduler's
    limit on processes it runs at once (hws_max_conc_proc; past it the firmware time-slices
    whole processes)."""
    out = {}
    base = "/sys/class/kfd/kfd/proc"
    try:
        procs = os.listdir(base)
        out["kfd_processes"] = len(procs)
        q = f"{base}/{os.getpid()}/queues"
        out["own_queues"] = len(os.listdir(q)) if os.path.isdir(q) else None
    except OSError:
        pass
    out["gpu_max_hw_queues"] = os.environ.get("GPU_MAX_HW_QUEUES")
    for prm in ("hws_max_conc_proc", "sched_policy", "mes", "cwsr_enable"):
        v = _read(f"/sys/module/amdgpu/parameters/{prm}")
        if v is not None:
            out[prm] = v
    return out


def cpu_seconds() -> float:
    import resource
    ru = resource.getrusage(resource.RUSAGE_SELF)
    return ru.ru_utime + ru.ru_stime


def measure(ctx, args, matrix, K, W, nloc, nnz_loc, world, barrier, allmax, gather=None):
    """W untimed + K timed fixed-length runs (rbl_start + m_max block steps, convergence checks
    off) on the matrix the context holds; the max over ranks of the timed region, the stage
    times (hipEvents) and the SpMM / partial-reorth rooflines priced from them.  On several
    ranks (`gather`: an all-gather of a Python object) every rank's own record as well: its
    run times, its stage split, its collectives (counts, bytes, host and device time per
    call), and the CPU time its process used against the CPUs it may run on."""
    import rbl
    from rbl import _lib
    n, b, k = args.n, args.b, args.k
    m_max = rbl.rbl_gpu.max_steps_for(args.kryl, b)
    spmm_kid = ctx.spmm_kernel_for(b)
    mat_fmt = ctx.matrix_format()
    spmm_kernel = {1: "gather", 2: "lds-window", 3: "lds-band-mfma", 5: "band-tile-mfma",
                   6: "segmented-gather", 7: "column-panel-csr"}[spmm_kid]

    host = {"start": 0.0, "enqueue": 0.0, "fetch_wait": 0.0}

    def one_run():
        _, _, info = rbl.lanczos(ctx, k, b, kryl_sz=args.kryl, seed=args.seed + 1, check=False,
                                 ritz=False, basis_bits=args.basis_bits)
        host["start"] += info.start_ms
        host["enqueue"] += info.enqueue_ms
        host["fetch_wait"] += info.fetch_ms

    for w_ in range(W):
        one_run()
        progress(f"{matrix} n={n} b={b}: warmup run {w_ + 1}/{W}")
    for key in host:
        host[key] = 0.0
    # the timed region records hipEvents only around the two kernels priced against their
    # rooflines (RBL_OPT_TIMERS 2: the SpMM's "AQ" and "part reorth" stages); every stage
    # boundary timed (1) is ~12 timestamped events per block step, a few us of queue time each,
    # so the full stage split comes from a second pass of the same K runs
    ctx.set_option(_lib.RBL_OPT_TIMERS, 2)
    barrier()
    ctx.synchronize()
    ctx.reset_timers()
    ctx.comm_stats(reset=True)
    barrier()
    cg0 = cgroup_cpu() if world > 1 else {}
    cpu0 = cpu_seconds()
    t0 = time.perf_counter()
    marks = [t0]
    for k_ in range(K):
        one_run()  # (returns once the run's last block step has been fetched)
        marks.append(time.perf_counter())
        progress(f"{matrix} n={n} b={b}: timed run {k_ + 1}/{K} {(marks[-1] - marks[-2]) * 1e3:.1f} ms")
    ctx.synchronize()
    local_elapsed = time.perf_counter() - t0
    local_cpu = cpu_seconds() - cpu0
    threads_timed = host_threads() if world > 1 else None
    cg1 = cgroup_cpu() if world > 1 else {}
    gpu_procs = gpu_processes() if world > 1 else {}
    barrier()
    elapsed = allmax(time.perf_counter() - t0)
    comm_full = ctx.comm_stats(times=True)
    comm = {k_: v for k_, v in comm_full.items() if not k_.endswith("_ns")}
    # the spread of the timed runs on this rank (rank 0's is reported): run-to-run variation
    runs_ms = sorted((b_ - a_) * 1e3 for a_, b_ in zip(marks, marks[1:]))
    run_spread = {"min": round(runs_ms[0], 2), "median": round(runs_ms[len(runs_ms) // 2], 2),
                  "max": round(runs_ms[-1], 2)} if runs_ms else None
    host_timed = dict(host)
    stage_timed = ctx.timers()  # "AQ" and "part reorth" of the timed region
    ctx.set_option(_lib.RBL_OPT_TIMERS, 1)
    barrier()
    ctx.synchronize()
    ctx.reset_timers()
    ctx.comm_stats(reset=True)
    barrier()
    t1 = time.perf_counter()
    for k_ in range(K):
        one_run()
        progress(f"{matrix} n={n} b={b}: stage-timer run {k_ + 1}/{K}")
    ctx.synchronize()
    local_staged = time.perf_counter() - t1
    barrier()
    elapsed_staged = allmax(time.perf_counter() - t1)
    comm_staged = ctx.comm_stats(times=True)
    host = host_timed
    stage = ctx.timers()
    per_rank = None
    if gather is not None and world > 1 and K:
        try:
            aff = len(os.sched_getaffinity(0))
        except (AttributeError, OSError):
            aff = os.cpu_count()
        calls_ar = max(1, comm_full["allreduce_calls"])
        calls_x = max(1, comm_full["exchange_calls"])
        mine = {
            "rank": int(os.environ.get("RANK", "0")), "device": ctx.device,
            "rows": int(nloc), "nnz": int(nnz_loc),
            "timed_ms_per_run": round(local_elapsed * 1e3 / K, 2),
            "run_ms_median": run_spread_median(marks),
            "stage_pass_ms_per_run": round(local_staged * 1e3 / K, 2),
            "stage_ms_per_run": {s_: round(v / K, 3) for s_, v in stage.items()},
            "host_ms_per_run": {key: round(v / K, 1) for key, v in host_timed.items()},
            "allreduce_calls_per_run": round(comm_full["allreduce_calls"] / K, 2),
            "allreduce_bytes_per_run": int(comm_full["allreduce_bytes"] / K),
            "exchange_calls_per_run": round(comm_full["exchange_calls"] / K, 2),
            "send_bytes_per_run": int(comm_full["send_bytes"] / K),
            "recv_bytes_per_run": int(comm_full["recv_bytes"] / K),
            # timed region: host wall time inside the transport calls
            "allreduce_host_us_per_call": round(comm_full["allreduce_host_ns"] / calls_ar / 1e3, 1),
            "exchange_host_us_per_call": round(comm_full["exchange_host_ns"] / calls_x / 1e3, 1),
            # stage pass: hipEvent span of each call on its stream (peers' lateness included)
            "allreduce_dev_us_per_call": round(comm_staged["allreduce_dev_ns"]
                                               / max(1, comm_staged["allreduce_calls"]) / 1e3, 1),
            "exchange_dev_us_per_call": round(comm_staged["exchange_dev_ns"]
                                              / max(1, comm_staged["exchange_calls"]) / 1e3, 1),
            "cpu_s_per_run": round(local_cpu / K, 3),
            "affinity_cpus": aff,
            "threads": threads_timed,
            "cgroup": {**{k_: cg1[k_] for k_ in ("quota_cpus",) if k_ in cg1},
                       **{f"{k_}_timed": cg1[k_] - cg0.get(k_, 0) for k_ in cg1
                          if k_ != "quota_cpus" and isinstance(cg1[k_], int)}},
            "gpu": gpu_procs,
        }
        per_rank = gather(mine)
    host = host_timed
    iters = K * m_max
    value = iters / elapsed
    stage_per_run = {s: v / K for s, v in stage.items()}

    # ---- roofline: SpMM (HBM) and partial reorth (fp64 MFMA), live from HIP events ----
    spmm_launches = K * (m_max + 1)               # rbl_start + one per block step
    spmm_ms = stage_timed["AQ"] / spmm_launches
    # algorithmic bytes: nnz*(8+4) + (n+1)*8 + read Q + write U
    # (+ read Q_{i-1} for the fused 3-term epilogue on the m_max step launches)
    bytes_step = nnz_loc * 12 + (nloc + 1) * 8 + 3 * nloc * b * 8
    bytes_start = nnz_loc * 12 + (nloc + 1) * 8 + 2 * nloc * b * 8
    # RBL_OPT_FUSE bit 2: the step launches from i = 2 on also apply the local reorth to the Q_i
    # rows they stage (Q_i and Q_{i-1} are read anyway) and write Q_i back: + n b 8 each
    lfused = bool(args.fuse & 4) and spmm_kid == 5 and b == 32 and args.basis_bits == 64 \
        and mat_fmt != 2
    spmm_bytes = (m_max * bytes_step + bytes_start + (m_max - 1) * nloc * b * 8 * lfused) / (m_max + 1)
    spmm_gbs = spmm_bytes / (spmm_ms * 1e-3) / 1e9
    reorth_flops = sum(8.0 * nloc * b * b * (i - 2) for i in range(4, m_max + 1, 2))
    reorth_ms = stage_timed["part reorth"] / K
    reorth_tf = reorth_flops / (reorth_ms * 1e-3) / 1e12 if reorth_ms > 0 else 0.0
    # HBM bytes from PMC counters (tools/pmc_traffic.sh -> tools/pmc_summarize.py; separate
    # FETCH_SIZE / WRITE_SIZE passes, gfx950 per-width calibration): a committed measurement of
    # the same kernels on the same config, used only when the config matches
    traffic = traffic_reorth = None
    fmt_name = {0: "csr", 1: "band tiles", 2: "packed band tiles", 3: "half band tiles", 4: "dense"}[mat_fmt]
    try:
        with open(args.traffic_json) as f:
            tj = json.load(f)
        for rec in [tj] + list(tj.get("workloads", [])):
            tc = rec.get("config", {})
            if (tc.get("n") == n and tc.get("b") == b and world == 1 and args.basis_bits == 64
                    and tc.get("matrix", "hashwindow") == matrix and tc.get("fuse") == args.fuse
                    and tc.get("matrix_format") == fmt_name):  # the same kernels as measured
                traffic = rec.get("spmm_hbm_bytes_per_launch")
                traffic_reorth = rec.get("part_reorth_hbm_bytes_per_run")
                break
    except (OSError, ValueError):
        pass
    roof_spmm = {"kernel": f"spmm {spmm_kernel} (AQ stage)", "bound": "hbm", "achieved": round(spmm_gbs, 1),
                 "peak": HBM_PEAK_GBS, "unit": "GB/s", "frac": round(spmm_gbs / HBM_PEAK_GBS, 4),
                 "traffic": None if traffic is None else int(traffic),
                 "algorithmic_bytes_per_launch": int(spmm_bytes),
                 "streamed_bytes_per_launch": int(streamed_bytes(spmm_kid, nloc, nnz_loc, b, args.halfwidth, m_max,
                                                                 mat_fmt)
                                                  + (m_max - 1) * nloc * b * 8 * lfused / (m_max + 1)),
                 "matrix_format": fmt_name,
                 # gather kernels (unbanded patterns) also read one Q row (b * 8 B) per nonzero,
                 # served by L2 / Infinity Cache / HBM: the traffic that bounds them
                 **({"q_row_gather_bytes_per_launch": int(nnz_loc * b * 8),
                     "gbs_incl_q_row_gathers": round((spmm_bytes + nnz_loc * b * 8) / (spmm_ms * 1e-3) / 1e9, 1)}
                    if spmm_kid in (1, 6) else {}),
                 "fused_local_reorth": lfused,
                 "ms_per_launch": round(spmm_ms, 4)}
    mfma_peak = FP64_MFMA_PEAK_TF if args.basis_bits == 64 else FP32_MFMA_PEAK_TF
    # the clock the chip holds under these kernels (profiles/pmc_clock.json: GRBM_GUI_ACTIVE
    # / 8 / wall, MI355X_MICROARCH.md 'DVFS give-back'): the spec peak assumes 2.4 GHz
    held = None
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_clock.json")) as f:
            kc = json.load(f)["kernels"]
        # the partial-reorth kernels at b = 32 (the Gram and the 64-column update, any variant)
        ks = [v for k_, v in kc.items() if k_.startswith(("k_gram44<32, 2", "k_tsmm44f<32"))]
        if ks and args.basis_bits == 64 and b == 32:
            held = sum(k["clock_ghz"] * k["avg_us"] for k in ks) / sum(k["avg_us"] for k in ks)
    except (OSError, ValueError, KeyError):
        pass
    # bytes (2m + 6) B_blk per even step (the basis read by the Gram and by the
    # update, plus the pair read / written); below the ridge (b = 16: AI ~ b/2) the stage is
    # HBM-bound and priced against the HBM peak instead
    s_basis = 8 if args.basis_bits == 64 else 4
    reorth_bytes = sum((2 * (i - 2) + 6) * nloc * b * s_basis for i in range(4, m_max + 1, 2))
    ai = reorth_flops / reorth_bytes if reorth_bytes else 0.0
    ridge = mfma_peak * 1e12 / (HBM_PEAK_GBS * 1e9)
    reorth_gbs = reorth_bytes / (reorth_ms * 1e-3) / 1e9 if reorth_ms > 0 else 0.0
    mbound = ai >= ridge
    roof_reorth = {"kernel": "partial reorth (gram+update)" + ("" if args.basis_bits == 64 else ", fp32"),
                   "bound": "mfma" if mbound else "hbm",
                   "achieved": round(reorth_tf, 2) if mbound else round(reorth_gbs, 1),
                   "peak": mfma_peak if mbound else HBM_PEAK_GBS,
                   "unit": "TFLOP/s" if mbound else "GB/s",
                   "frac": round(reorth_tf / mfma_peak if mbound else reorth_gbs / HBM_PEAK_GBS, 4),
                   "arithmetic_intensity": round(ai, 2), "ridge": round(ridge, 2),
                   "algorithmic_bytes_per_run": int(reorth_bytes),
                   "tflops": round(reorth_tf, 2),
                   "traffic": None if traffic_reorth is None else int(traffic_reorth),
                   "traffic_unit": f"HBM bytes per run (gram + update, {len(range(4, m_max + 1, 2))} launches each)",
                   "algorithmic_flops_per_run": reorth_flops, "ms_per_run": round(reorth_ms, 3),
                   **({"held_clock_ghz": round(held, 3),
                       "frac_of_peak_at_held_clock": round(reorth_tf / (mfma_peak * held / 2.4), 4)}
                      if held and mbound else {})}
    if stage_timed["part reorth"] > stage_timed["AQ"]:
        roofline, roofline2 = roof_reorth, roof_spmm
    else:
        roofline, roofline2 = roof_spmm, roof_reorth
    # collectives per block step on this rank (all-reduces, grouped send/recv), from the library
    steps_timed = K * (m_max + 1)
    # (the halo-plan entries of rbl_comm_stats are per matrix, not counters: the R-MAT
    # sub-record reports them as halo_plan)
    plan_keys = ("halo_push", "push_rows_pred", "pull_rows_pred")
    comm_per_step = {key: round(v / steps_timed, 3) for key, v in comm.items()
                     if key not in plan_keys}
    # the host side of a run (rbl.lanczos): rbl_start (blocks until A Omega + QR are done),
    # enqueueing the steps, and waiting in rbl_fetch for the last one
    host_ms = {key: round(v / K, 1) for key, v in host.items()}
    return {"elapsed": elapsed, "stage": stage, "value": value, "roofline": roofline,
            "per_rank": per_rank,
            "host_ms_per_run": host_ms,
            "stage_pass_ms_per_run": round(elapsed_staged * 1e3 / K, 2) if K else None,
            "roofline_secondary": roofline2, "spmm_kernel": spmm_kernel,
            "comm_per_step": comm_per_step, "m_max": m_max, "run_ms": run_spread}


def run_spread_median(marks) -> float:
    runs = sorted((b_ - a_) * 1e3 for a_, b_ in zip(marks, marks[1:]))
    return round(runs[len(runs) // 2], 2) if runs else 0.0


def rank_arrays(per_rank):
    """The ranks' own records as arrays indexed by rank (the multi-rank line's self-diagnosis):
    each rank's stage split of the stage pass and what it leaves unattributed (host gaps: the
    stream idle while the host enqueues or waits), its collectives' per-call host and device
    times, its bytes, and the CPU time its process used — with the job's total CPU time per
    wall second against the CPUs the ranks may run on (>= ~0.9: the host is saturated, and every
    host-side step of every rank waits for a core)."""
    if not per_rank:
        return None
    per_rank = sorted(per_rank, key=lambda r: r["rank"])
    stages = list(per_rank[0]["stage_ms_per_run"])
    out = {"ranks": [r["rank"] for r in per_rank], "devices": [r["device"] for r in per_rank]}
    for key in ("rows", "nnz", "timed_ms_per_run", "run_ms_median", "stage_pass_ms_per_run",
                "allreduce_calls_per_run", "allreduce_bytes_per_run", "exchange_calls_per_run",
                "send_bytes_per_run", "recv_bytes_per_run", "allreduce_host_us_per_call",
                "exchange_host_us_per_call", "allreduce_dev_us_per_call",
                "exchange_dev_us_per_call", "cpu_s_per_run"):
        out[key] = [r[key] for r in per_rank]
    out["stage_ms_per_run"] = {s_: [r["stage_ms_per_run"][s_] for r in per_rank] for s_ in stages}
    sums = [round(sum(r["stage_ms_per_run"].values()), 2) for r in per_rank]
    out["stage_sum_ms"] = sums
    out["stage_sum_over_run"] = [round(sm / r["stage_pass_ms_per_run"], 4) if r["stage_pass_ms_per_run"] else None
                                 for sm, r in zip(sums, per_rank)]
    out["unattributed_ms"] = [round(r["stage_pass_ms_per_run"] - sm, 2) for sm, r in zip(sums, per_rank)]
    out["host_ms_per_run"] = {key: [r["host_ms_per_run"][key] for r in per_rank]
                              for key in per_rank[0]["host_ms_per_run"]}
    aff = max(r["affinity_cpus"] or 1 for r in per_rank)
    cpu_total = sum(r["cpu_s_per_run"] for r in per_rank)
    wall = max(r["timed_ms_per_run"] for r in per_rank) / 1e3
    out["host_cpu"] = {"affinity_cpus": aff, "os_cpu_count": os.cpu_count(),
                       "cpu_s_per_run_all_ranks": round(cpu_total, 3),
                       "busy_cpus": round(cpu_total / wall, 2) if wall else None,
                       "saturation": round(cpu_total / wall / aff, 3) if wall else None,
                       "threads_rank0": per_rank[0]["threads"],
                       "threads_per_rank": [sum((r["threads"] or {}).values()) for r in per_rank],
                       # the cgroup's quota and its throttling over rank 0's timed region
                       "cgroup_rank0": per_rank[0].get("cgroup")}
    out["gpu_processes"] = {"rank0": per_rank[0].get("gpu"),
                            "queues_per_rank": [(r.get("gpu") or {}).get("own_queues") for r in per_rank]}
    busiest = max(range(len(per_rank)), key=lambda i: per_rank[i]["stage_pass_ms_per_run"])
    out["slowest_rank"] = per_rank[busiest]["rank"]
    return out


# DESIGN §6's prediction for the driver's curve (block-iters/s, one MI355X per rank over xGMI):
# per-rank compute = the N = 1 run / N, plus ~30 us per all-reduce and the halo per SpMM
SCALING_MODEL = {"C4a hash-window SpMM-Lanczos": {1: 46.83, 2: 92.0, 4: 181.0, 8: 350.0},
                 "C4b R-MAT SpMM-Lanczos": {1: 18.05, 2: 33.0, 4: 63.0, 8: 125.0}}


def model_block(workload, world, value, shared_gpu):
    """The §6 model's value for this N and workload beside the measured one.  When the ranks
    share GPUs (a one-GPU rehearsal) the xGMI prediction does not apply: the ranks split one
    GPU's time, so the expectation is the N = 1 value (the same total work), and the ratio
    measures what sharing and the loopback transport cost."""
    m = SCALING_MODEL.get(workload)
    if not m:
        return None
    out = {"source": "DESIGN.md §6 (modelled, not measured): per-rank compute = N=1 run time / N, "
                     "~30 us per RCCL all-reduce, halo bytes over the xGMI links (~55 GB/s each)",
           "n_gpus": world, "predicted_xgmi": m.get(world)}
    if shared_gpu:
        out.update({"applies": False, "shared_gpu_expectation": m[1],
                    "measured_over_shared_gpu_expectation": round(value / m[1], 3)})
    elif m.get(world):
        out.update({"applies": True, "measured_over_predicted": round(value / m[world], 3)})
    return out


def main():
    args = parse()
    launch_ranks(args)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    # stdout carries the one JSON line and nothing else: what libraries print there (gloo's
    # connection notes, RCCL's banner and warnings) goes to stderr from here on
    sys.stdout.flush()
    line_fd = os.dup(1)
    os.dup2(2, 1)
    dist = None
    if world > 1:
        import torch.distributed as dist
        dist.init_process_group("gloo")

    def barrier():
        if dist is not None:
            dist.barrier()

    def allmax(x: float) -> float:
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def allsum(x: int) -> int:
        if dist is None:
            return x
        import torch
        t = torch.tensor([x], dtype=torch.int64)
        dist.all_reduce(t)
        return int(t.item())

    def gather_obj(x) -> list:
        if dist is None:
            return [x]
        out = [None] * world
        dist.all_gather_object(out, x)
        return out

    def allgather_i64(x: int) -> list:
        if dist is None:
            return [int(x)]
        import torch
        out = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(out, torch.tensor([int(x)], dtype=torch.int64))
        return [int(t.item()) for t in out]

    import rbl
    from rbl import _lib
    uid = None
    shm_path = None
    device = local_rank
    ngpu = gpu_count_sysfs() or 1
    # a one-GPU rehearsal (shm transport, or RCCL with a host id per rank): ranks share GPUs
    shared_gpu = (args.transport == "shm" or rccl_host_per_rank()) and world > ngpu
    if world > 1 and args.transport == "shm":
        # one segment per job, named by rank 0; ranks beyond the GPU count share GPUs
        import uuid
        obj = [f"/dev/shm/rbl_bench_{os.getpid()}_{uuid.uuid4().hex[:12]}" if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        shm_path = obj[0]
        device = local_rank % ngpu
    elif world > 1:
        if rccl_host_per_rank():  # one-GPU rehearsal of the RCCL path (see rccl_host_per_rank)
            os.environ["NCCL_HOSTID"] = f"rbl-bench-host-{rank}"
            os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
            device = local_rank % ngpu
        buf = np.zeros(128, np.uint8)
        if rank == 0:
            st = _lib.lib.rbl_get_unique_id(_lib.u8ptr(buf))
            assert st == 0, "rbl_get_unique_id failed"
        obj = [bytes(buf)]
        dist.broadcast_object_list(obj, src=0)
        uid = obj[0]
    ctx = rbl.Context(device, nranks=world, rank=rank, unique_id=uid, shm_path=shm_path)

    n, b, k = args.n, args.b, args.k
    ctx.set_option(_lib.RBL_OPT_KEEP_CSR, args.keep_csr)
    plant = np.array([100.0 * (2 * k + 1 - l) for l in range(1, 2 * k + 1)])
    t0 = time.perf_counter()
    if args.matrix == "rmat":
        if not args.rmat_edges:
            args.rmat_edges = int(0.66 * 100 * n)
        ctx.set_option(_lib.RBL_OPT_RELABEL, rmat_relabel(args, world))
        ctx.gen_rmat(n, args.rmat_scale, args.rmat_edges, args.seed, plant)
    elif args.matrix == "circuit":
        ctx.gen_circuit(n, args.seed, plant)
    else:
        ctx.gen_hashwindow(n, args.halfwidth, args.density, args.seed, plant)
    gen_s = time.perf_counter() - t0
    progress(f"{args.matrix} matrix generated ({gen_s:.1f} s)")
    _, r0, r1, nnz_loc = ctx.matrix_info()
    nloc = r1 - r0
    nnz = allsum(nnz_loc)
    ctx.set_option(_lib.RBL_OPT_TIMERS, 1)
    ctx.set_option(_lib.RBL_OPT_SPMM_KERNEL, args.spmm_kernel)
    ctx.set_option(_lib.RBL_OPT_DEVICE_BLOCKS, args.device_blocks)
    ctx.set_option(_lib.RBL_OPT_FUSE, args.fuse)
    m_max = rbl.rbl_gpu.max_steps_for(args.kryl, b)
    meas = measure(ctx, args, args.matrix, args.steps, args.warmup, nloc, nnz_loc, world,
                   barrier, allmax, gather_obj)
    K = args.steps
    elapsed, stage, value = meas["elapsed"], meas["stage"], meas["value"]
    stage_per_run = {s: v / K for s, v in stage.items()}
    roofline, roofline2 = meas["roofline"], meas["roofline_secondary"]

    # ---- time-to-k (convergence on, start -> converged Ritz vectors) ----
    progress("time-to-k")
    ttk = None
    if not args.no_ttk:
        barrier()
        ctx.synchronize()
        ctx.reset_timers()
        t0 = time.perf_counter()
        D, V, info = rbl.lanczos(ctx, k, b, kryl_sz=args.kryl, seed=args.seed + 2, check=True,
                                 ritz=True, basis_bits=args.basis_bits,
                                 speculate=args.speculate == "auto" and "auto")
        ctx.synchronize()
        barrier()
        ttk_s = allmax(time.perf_counter() - t0)
        ttk_stage = ctx.timers()
        ttk = {"seconds": round(ttk_s, 4), "iters": info.iters, "converged": info.converged,
               "k": k, "top_eigenvalues": [round(float(x), 6) for x in D[:3]],
               "ritz_ms": round(allmax(ttk_stage["Ritz vectors"]), 3),
               "host_eig_ms": round(info.eig_ms, 3),
               "host_ms": {"start": round(info.start_ms, 1), "fetch_wait": round(info.fetch_ms, 1),
                           "eig": round(info.eig_ms, 1), "ritz_and_d2h": round(info.ritz_ms, 1)},
               "stage_ms": {s_: round(v, 3) for s_, v in ttk_stage.items()},
               "speculated_steps": info.spec_steps, "speculated_discarded": info.spec_wasted}

    # ---- time-to-k on a slowly decaying spectrum (same generator and n, another plant) ----
    ttk_slow = None
    if not args.no_ttk and not args.no_ttk_slow and args.matrix == "hashwindow":
        slow_plant = np.array([12.0 + 0.25 * (2 * k + 1 - l) for l in range(1, 2 * k + 1)])
        ctx.gen_hashwindow(n, args.halfwidth, args.density, args.seed, slow_plant)
        # one untimed start + step on the run's own plan (m_max blocks, so the timed run reuses
        # every allocation) builds the band tiles and run buffers of the new matrix
        ctx.start(b, m_max, seed=args.seed + 2, basis_bits=args.basis_bits)
        ctx.step(1, False)
        # the planted run's 1.6 GB of Ritz vectors are released here, not by the assignment
        # below inside the timed region (unmapping them took ~20 ms of it)
        V = None
        barrier()
        ctx.synchronize()
        ctx.reset_timers()
        t0 = time.perf_counter()
        D, V, info = rbl.lanczos(ctx, k, b, kryl_sz=args.kryl, seed=args.seed + 2, check=True,
                                 ritz=True, basis_bits=args.basis_bits,
                                 speculate=args.speculate == "auto" and "auto")
        ctx.synchronize()
        barrier()
        ts = allmax(time.perf_counter() - t0)
        st_ = ctx.timers()
        ttk_slow = {"seconds": round(ts, 4), "iters": info.iters, "converged": info.converged,
                    "k": k, "spectrum": "planted 12 + 0.25 (2k+1-l), l = 1..2k",
                    "top_eigenvalues": [round(float(x), 6) for x in D[:3]],
                    "kth_eigenvalue": round(float(D[k - 1]), 6),
                    "host_eig_ms": round(info.eig_ms, 3),
                    "host_ms": {"start": round(info.start_ms, 1), "fetch_wait": round(info.fetch_ms, 1),
                                "eig": round(info.eig_ms, 1), "ritz_and_d2h": round(info.ritz_ms, 1)},
                    "stage_ms": {s_: round(v, 3) for s_, v in st_.items()},
                    "speculated_steps": info.spec_steps, "speculated_discarded": info.spec_wasted,
                    "max_residual_per_check": [float("%.3g" % r) for r in info.resid]}

    # ---- BASELINE config 4 (C4b): the R-MAT pattern at the same n, b, k, same ranks ----
    # A sub-record that raises on one rank leaves the headline line unprinted; on one rank
    # (no collectives in flight) the error is recorded in the sub-record instead.  On several
    # ranks it propagates, so torch.distributed.run ends the peers instead of leaving them
    # waiting in a collective — except a run that could not allocate its buffers: rbl_start
    # votes on that before its collectives, so every rank raises it together and all record it.
    def guarded(fn, *a):
        try:
            return fn(*a)
        except Exception as e:  # noqa: BLE001 — reported in the line
            collective = (isinstance(e, rbl.RBLError) and e.code == _lib.RBL_ERR_OOM
                          and "rbl_start" in str(e))
            if world > 1 and not collective:
                raise
            return {"error": f"{type(e).__name__}: {e}"}

    rmat_rec = None
    if args.matrix == "hashwindow" and args.rmat_steps > 0 and args.basis_bits == 64:
        progress("C4b sub-record")
        rmat_rec = guarded(rmat_subrecord, ctx, args, plant, world, barrier, allmax, allsum,
                           allgather_i64, gather_obj, shared_gpu)

    # ---- BASELINE config 3's shape: the circuit-like matrix at G3_circuit's n, b = 16 ----
    c3_rec = None
    if args.matrix == "hashwindow" and args.c3_steps > 0 and args.basis_bits == 64:
        progress("C3 sub-record")
        c3_rec = guarded(c3_subrecord, ctx, args, world, barrier, allmax, allsum, allgather_i64,
                         gather_obj)

    # ---- a wide band (the FEM / circuit orderings benchmark.jl loads): the column panels ----
    wide_rec = None
    if args.matrix == "hashwindow" and args.wide_steps > 0 and args.basis_bits == 64 and args.b == 32:
        progress("wide-band sub-record")
        wide_rec = guarded(wide_subrecord, ctx, args, plant, world, barrier, allmax, allsum,
                           allgather_i64, gather_obj)

    # ---- CPU baseline: the oracle (port of RBL.jl) on a bounded sample, rank 0, N = 1 ----
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        progress("CPU baseline")
        cpu = cpu_baseline(args, m_max, plant)

    comm = ctx.comm_info()
    nnz_ranks = allgather_i64(nnz_loc)
    # the line is complete but for C5 before C5 runs: a C5 failure on this rank still prints it
    # (with the error in c5_mixed) before the job ends non-zero
    line = {
        "metric": metric_name(args, nnz),
        "value": round(value, 3),
        "unit": "block iterations/s",
        "n_gpus": world if args.transport == "rccl" and not rccl_host_per_rank() else min(world, ngpu),
        "steps": K,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed / K * 1e3, 3),
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "f64" if args.basis_bits == 64 else "f64 (A*Q, 3-term, QR) + f32 (basis, reorth)",
        "data": f"synthetic (seeded {args.matrix} symmetric matrix generated on device)",
        "config": {"workload": workload_name(args),
                   "n": n, "nnz": nnz, "b": b, "k": k, "matrix": args.matrix,
                   **({"halfwidth": args.halfwidth, "density": args.density}
                      if args.matrix == "hashwindow" else
                      {"rmat_scale": args.rmat_scale, "rmat_edges": args.rmat_edges,
                       "rmat_abcd": [0.57, 0.19, 0.19, 0.05],
                       "relabel": bool(rmat_relabel(args, world))} if args.matrix == "rmat" else
                      {"circuit_width": 1259, "circuit_p_edge": 0.95873}),
                   "block_steps_per_run": m_max, "parallelism": f"rows{world}",
                   "transport": comm["transport"], "transport_ranks": comm["nranks"],
                   **({"rccl_version": comm["rccl_version"], "rccl_path": comm["rccl_path"]}
                      if comm["transport"] == "rccl" else {}),
                   **({"ranks_share_gpus": True, "gpus_used": min(world, ngpu)}
                      if (args.transport == "shm" or rccl_host_per_rank()) and world > ngpu
                      else {}),
                   **({"rccl_host_per_rank": True} if rccl_host_per_rank() and world > 1
                      else {}),
                   "nnz_per_rank": nnz_ranks,
                   **({"device_blocks": args.device_blocks} if args.device_blocks else {}),
                   **({"keep_csr": 0} if not args.keep_csr else {}),
                   **({"fuse": args.fuse} if args.fuse != 7 else {})},
        "roofline": roofline,
        "roofline_secondary": roofline2,
        "stage_ms_per_run": {s: round(v, 3) for s, v in stage_per_run.items()},
        "host_ms_per_run": meas["host_ms_per_run"],
        # the same K runs again with the stage timers on (stage_ms_per_run and the rooflines)
        "stage_pass_ms_per_run": meas["stage_pass_ms_per_run"],
        "time_to_k": ttk,
        "time_to_k_slow_spectrum": ttk_slow,
        "matrix_gen_s": round(gen_s, 3),
        "cpu_baseline": cpu,
        "comm_per_step": meas["comm_per_step"], "run_ms_rank0": meas["run_ms"],
        # several ranks: every rank's own record (arrays by rank) and the §6 model's value
        **({"per_rank": rank_arrays(meas["per_rank"]),
            "model": model_block(workload_name(args), world, value, shared_gpu)}
           if world > 1 else {}),
        "c4b_rmat": rmat_rec,
        "c3_circuit": c3_rec,
        "c4w_wideband": wide_rec,
        "c5_mixed": None,
    }

    def emit():
        if rank == 0:
            out = (json.dumps(line) + "\n").encode()
            while out:
                out = out[os.write(line_fd, out):]

    # ---- BASELINE config 5: n = 5e7, fp32 basis, on >= 2 ranks (no spill) ----
    if (args.matrix == "hashwindow" and args.c5_steps > 0 and args.basis_bits == 64
            and world >= args.c5_min_ranks):
        progress("C5 sub-record")
        try:
            line["c5_mixed"] = guarded(c5_subrecord, ctx, args, world, barrier, allmax, allsum,
                                       allgather_i64)
        except Exception as e:  # noqa: BLE001 — a rank-local failure: report, then end non-zero
            line["c5_mixed"] = {"error": f"{type(e).__name__}: {e}", "rank": rank}
            emit()
            raise
    emit()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def rmat_subrecord(ctx, args, plant, world, barrier, allmax, allsum, allgather_i64,
                   gather_obj=None, shared_gpu=False):
    """BASELINE config 4 in the same driver run: the seeded R-MAT matrix
    ((a,b,c,d) = (0.57,0.19,0.19,0.05), scale 24, 0.66 n x 100 draws: ~1e9 nonzeros at n = 1e7)
    generated on the device in place of the headline matrix, nnz-balanced over the ranks; the
    same fixed-length runs (`args.rmat_warmup` untimed + `args.rmat_steps` timed, max over
    ranks), the SpMM priced on SURVEY's CSR bytes and on the Q-row gathers that bound it, and
    a time-to-k on its planted spectrum."""
    import copy
    import rbl
    ra = copy.copy(args)
    ra.matrix = "rmat"
    from rbl import _lib
    edges = args.rmat_edges or int(0.66 * 100 * args.n)
    relabel = rmat_relabel(args, world)
    ctx.set_option(_lib.RBL_OPT_RELABEL, relabel)
    ctx.set_option(_lib.RBL_OPT_HALO_PUSH, args.halo_push)
    t0 = time.perf_counter()
    ctx.gen_rmat(args.n, args.rmat_scale, edges, args.seed, plant)
    ctx.set_option(_lib.RBL_OPT_RELABEL, 0)
    gen_s = time.perf_counter() - t0
    plan = ctx.comm_stats()
    _, r0, r1, nnz_loc = ctx.matrix_info()
    nloc = r1 - r0
    nnz = allsum(nnz_loc)
    meas = measure(ctx, ra, "rmat", args.rmat_steps, args.rmat_warmup, nloc, nnz_loc, world,
                   barrier, allmax, gather_obj)
    K = args.rmat_steps
    barrier()
    ctx.synchronize()
    ctx.reset_timers()
    t0 = time.perf_counter()
    D, V, info = rbl.lanczos(ctx, args.k, args.b, kryl_sz=args.kryl, seed=args.seed + 2,
                             check=True, ritz=True)
    ctx.synchronize()
    barrier()
    ttk_s = allmax(time.perf_counter() - t0)
    # the relabelled matrix is P A P^T of the one drawn: the as-drawn matrix measured beside it
    # keeps the line comparable with the rounds before the relabel (round 3: 16.95)
    as_drawn = None
    if relabel and args.rmat_as_drawn_steps > 0:
        ctx.gen_rmat(args.n, args.rmat_scale, edges, args.seed, plant)
        _, r0d, r1d, nnz_d = ctx.matrix_info()
        md = measure(ctx, ra, "rmat", args.rmat_as_drawn_steps, 1, r1d - r0d, nnz_d, world,
                     barrier, allmax)
        as_drawn = {"value": round(md["value"], 3), "unit": "block iterations/s",
                    "steps": args.rmat_as_drawn_steps, "warmup": 1,
                    "ms_per_step": round(md["elapsed"] / args.rmat_as_drawn_steps * 1e3, 3),
                    "spmm_ms_per_launch": next(r_["ms_per_launch"] for r_ in
                                               (md["roofline"], md["roofline_secondary"])
                                               if r_["kernel"].startswith("spmm")),
                    "nnz_per_rank": allgather_i64(nnz_d)}
    return {"workload": "C4b R-MAT SpMM-Lanczos" if (args.n, args.b) == (10_000_000, 32)
            else "R-MAT SpMM-Lanczos",
            "metric": f"RBL iters/sec, n={args.n:.0e} nnz/row={nnz / args.n:.0f} b={args.b} (rmat)",
            "value": round(meas["value"], 3), "unit": "block iterations/s",
            "steps": K, "warmup": args.rmat_warmup,
            "ms_per_step": round(meas["elapsed"] / K * 1e3, 3),
            "n": args.n, "nnz": nnz, "rmat_scale": args.rmat_scale, "rmat_edges": edges,
            "rmat_abcd": [0.57, 0.19, 0.19, 0.05], "nnz_per_rank": allgather_i64(nnz_loc),
            "relabel": bool(relabel),
            "halo_plan": {"push_pull_split": bool(plan["halo_push"]),
                          "rows_per_spmm_split": plan["push_rows_pred"],
                          "rows_per_spmm_pull_all": plan["pull_rows_pred"]},
            "send_bytes_per_step_by_rank": allgather_i64(int(meas["comm_per_step"]["send_bytes"])),
            "roofline": meas["roofline"], "roofline_secondary": meas["roofline_secondary"],
            "stage_ms_per_run": {s_: round(v / K, 3) for s_, v in meas["stage"].items()},
            "comm_per_step": meas["comm_per_step"], "run_ms_rank0": meas["run_ms"],
            **({"per_rank": rank_arrays(meas["per_rank"]),
                "model": model_block("C4b R-MAT SpMM-Lanczos" if (args.n, args.b) == (10_000_000, 32)
                                     else None, world, meas["value"], shared_gpu)}
               if world > 1 else {}),
            "time_to_k": {"seconds": round(ttk_s, 4), "iters": info.iters,
                          "converged": info.converged, "k": args.k,
                          "top_eigenvalues": [round(float(x), 6) for x in D[:3]]},
            "matrix_gen_s": round(gen_s, 3),
            **({"as_drawn": as_drawn} if as_drawn else {})}


def c3_subrecord(ctx, args, world, barrier, allmax, allsum, allgather_i64, gather_obj=None):
    """BASELINE config 3's shape in the same driver run: the seeded
    circuit-like SPD matrix of G3_circuit's size (n = 1,585,478, 7.66 M nonzeros, scattered: no
    band; the real G3_circuit is not in the image) generated on the device, b = 16, k = 20; the
    same fixed-length runs (m_max = 75 steps at b = 16) and a time-to-k."""
    import copy
    import rbl
    ra = copy.copy(args)
    ra.matrix, ra.n, ra.b, ra.k = "circuit", 1_585_478, 16, 20
    plant = np.array([100.0 * (2 * ra.k + 1 - l) for l in range(1, 2 * ra.k + 1)])
    t0 = time.perf_counter()
    ctx.gen_circuit(ra.n, ra.seed, plant)
    gen_s = time.perf_counter() - t0
    _, r0, r1, nnz_loc = ctx.matrix_info()
    nloc = r1 - r0
    nnz = allsum(nnz_loc)
    K = args.c3_steps
    meas = measure(ctx, ra, "circuit", K, 1, nloc, nnz_loc, world, barrier, allmax, gather_obj)
    barrier()
    ctx.synchronize()
    ctx.reset_timers()
    t0 = time.perf_counter()
    D, V, info = rbl.lanczos(ctx, ra.k, ra.b, kryl_sz=ra.kryl, seed=ra.seed + 2, check=True,
                             ritz=True)
    ctx.synchronize()
    barrier()
    ttk_s = allmax(time.perf_counter() - t0)
    return {"workload": "C3-shaped circuit SpMM-Lanczos (G3_circuit's n and nnz, synthetic)",
            "metric": f"RBL iters/sec, n={ra.n} nnz/row={nnz / ra.n:.2f} b={ra.b} (circuit)",
            "value": round(meas["value"], 3), "unit": "block iterations/s",
            "steps": K, "warmup": 1, "ms_per_step": round(meas["elapsed"] / K * 1e3, 3),
            "n": ra.n, "nnz": nnz, "b": ra.b, "k": ra.k, "block_steps_per_run": meas["m_max"],
            "nnz_per_rank": allgather_i64(nnz_loc),
            "roofline": meas["roofline"], "roofline_secondary": meas["roofline_secondary"],
            "stage_ms_per_run": {s_: round(v / K, 3) for s_, v in meas["stage"].items()},
            "comm_per_step": meas["comm_per_step"], "run_ms_rank0": meas["run_ms"],
            **({"per_rank": rank_arrays(meas["per_rank"])} if world > 1 else {}),
            "time_to_k": {"seconds": round(ttk_s, 4), "iters": info.iters,
                          "converged": info.converged, "k": ra.k,
                          "top_eigenvalues": [round(float(x), 6) for x in D[:3]]},
            "matrix_gen_s": round(gen_s, 3)}


def wide_subrecord(ctx, args, plant, world, barrier, allmax, allsum, allgather_i64, gather_obj=None):
    """A wide band in the same driver run: the headline's generator at the same n and ~100
    nonzeros per row, but half-width --wide-halfwidth (default 1024, density 99 / 2H) — the regime
    of the FEM / circuit orderings the reference's benchmark.jl:21-28 loads, past the band tiles'
    64 — where the SpMM is the column-panel kernel (spmm_panel.hip); the same fixed-length runs
    and a time-to-k."""
    import copy
    import rbl
    ra = copy.copy(args)
    ra.halfwidth = args.wide_halfwidth
    ra.density = round(99.0 / (2 * ra.halfwidth), 6)
    t0 = time.perf_counter()
    ctx.gen_hashwindow(ra.n, ra.halfwidth, ra.density, ra.seed, plant)
    gen_s = time.perf_counter() - t0
    _, r0, r1, nnz_loc = ctx.matrix_info()
    nloc = r1 - r0
    nnz = allsum(nnz_loc)
    K = args.wide_steps
    meas = measure(ctx, ra, "hashwindow", K, 1, nloc, nnz_loc, world, barrier, allmax, gather_obj)
    barrier()
    ctx.synchronize()
    ctx.reset_timers()
    t0 = time.perf_counter()
    D, V, info = rbl.lanczos(ctx, ra.k, ra.b, kryl_sz=ra.kryl, seed=ra.seed + 3, check=True,
                             ritz=True)
    ctx.synchronize()
    barrier()
    ttk_s = allmax(time.perf_counter() - t0)
    return {"workload": f"wide-band hash-window SpMM-Lanczos (half-width {ra.halfwidth})",
            "metric": f"RBL iters/sec, n={ra.n} nnz/row={nnz / ra.n:.1f} b={ra.b} (hashwindow, "
                      f"halfwidth {ra.halfwidth})",
            "value": round(meas["value"], 3), "unit": "block iterations/s",
            "steps": K, "warmup": 1, "ms_per_step": round(meas["elapsed"] / K * 1e3, 3),
            "n": ra.n, "nnz": nnz, "b": ra.b, "k": ra.k, "halfwidth": ra.halfwidth,
            "density": ra.density, "block_steps_per_run": meas["m_max"],
            "nnz_per_rank": allgather_i64(nnz_loc),
            "roofline": meas["roofline"], "roofline_secondary": meas["roofline_secondary"],
            "stage_ms_per_run": {s_: round(v / K, 3) for s_, v in meas["stage"].items()},
            "comm_per_step": meas["comm_per_step"], "run_ms_rank0": meas["run_ms"],
            **({"per_rank": rank_arrays(meas["per_rank"])} if world > 1 else {}),
            "time_to_k": {"seconds": round(ttk_s, 4), "iters": info.iters,
                          "converged": info.converged, "k": ra.k,
                          "top_eigenvalues": [round(float(x), 6) for x in D[:3]]},
            "matrix_gen_s": round(gen_s, 3)}


def c5_subrecord(ctx, args, world, barrier, allmax, allsum, allgather_i64):
    """BASELINE config 5 in the same driver run: the hash-window matrix at
    n = 5e7 (~5e9 nonzeros, int64 row pointers), b = 32, k = 20, with the fp32 Krylov basis (the
    reference run with FLOAT = Float32: blocks and their reorth fp32, A*Q / 3-term / QR fp64),
    the CSR released once the band tiles exist (RBL_OPT_KEEP_CSR = 0), on >= 2 ranks so the
    basis (243 GB in fp32) stays in HBM; 1 untimed + `args.c5_steps` timed fixed-length runs and
    a time-to-k.  It replaces the headline matrix (the last sub-record)."""
    import copy
    import rbl
    from rbl import _lib
    ra = copy.copy(args)
    ra.n, ra.basis_bits, ra.keep_csr = args.c5_n, 32, 0
    plant = np.array([100.0 * (2 * ra.k + 1 - l) for l in range(1, 2 * ra.k + 1)])
    # every rank checks its HBM first and all skip together (a rank failing inside a collective
    # would leave its peers waiting): per local row ~2.4 KB while the matrix is built (CSR + band
    # tiles) and ~6.9 KB during the run (39 fp32 basis slots, band tiles, fp64 working blocks)
    nloc_est = -(-ra.n // world)
    need = 1.15 * nloc_est * max(2.4e3, 39 * 32 * 4 + 1152 + 3 * 256 + 64)
    # ranks sharing one GPU (the shm transport on a one-GPU box) all draw on its free memory
    devs = allgather_i64(ctx.device)
    need *= sum(1 for d in devs if d == ctx.device)
    free, total = ctx.device_memory()  # (the C3 matrix and its ~16 GB of buffers still held)
    if allsum(int(free < need)) > 0:
        return {"skipped": f"needs ~{need / 1e9:.0f} GB of HBM per rank; a rank has "
                           f"{free / 1e9:.0f} GB free"}
    ctx.set_option(_lib.RBL_OPT_KEEP_CSR, 0)
    t0 = time.perf_counter()
    ctx.gen_hashwindow(ra.n, ra.halfwidth, ra.density, ra.seed, plant)
    gen_s = time.perf_counter() - t0
    _, r0, r1, nnz_loc = ctx.matrix_info()
    nloc = r1 - r0
    nnz = allsum(nnz_loc)
    K = args.c5_steps
    meas = measure(ctx, ra, "hashwindow", K, 1, nloc, nnz_loc, world, barrier, allmax)
    barrier()
    ctx.synchronize()
    ctx.reset_timers()
    t0 = time.perf_counter()
    D, V, info = rbl.lanczos(ctx, ra.k, ra.b, kryl_sz=ra.kryl, seed=ra.seed + 2, check=True,
                             ritz=True, basis_bits=32)
    ctx.synchronize()
    barrier()
    ttk_s = allmax(time.perf_counter() - t0)
    return {"workload": "C5 hash-window SpMM-Lanczos, mixed precision (fp32 basis)",
            "metric": f"RBL iters/sec, n={ra.n:.0e} nnz/row={nnz / ra.n:.0f} b={ra.b} fp32 basis",
            "value": round(meas["value"], 3), "unit": "block iterations/s",
            "steps": K, "warmup": 1, "ms_per_step": round(meas["elapsed"] / K * 1e3, 3),
            "n": ra.n, "nnz": nnz, "b": ra.b, "k": ra.k, "keep_csr": 0,
            "nnz_per_rank": allgather_i64(nnz_loc),
            "roofline": meas["roofline"], "roofline_secondary": meas["roofline_secondary"],
            "stage_ms_per_run": {s_: round(v / K, 3) for s_, v in meas["stage"].items()},
            "comm_per_step": meas["comm_per_step"], "run_ms_rank0": meas["run_ms"],
            "time_to_k": {"seconds": round(ttk_s, 4), "iters": info.iters,
                          "converged": info.converged, "k": ra.k,
                          "top_eigenvalues": [round(float(x), 6) for x in D[:3]]},
            "matrix_gen_s": round(gen_s, 3)}


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


CPU_FIXED_START_BY_S = 240


def cpu_baseline(args, m_max, plant):
    """Time the oracle (NumPy/SciPy restatement of RBL.jl) on n_s rows of the same generator
    for the same m_max fixed block steps (measured end to end, matrix generation excluded), and
    scale its per-iteration time linearly to n (every stage of a block step is O(n) at fixed b
    and m).  With --cpu-one-thread the same sample runs again at 1 BLAS thread, as the
    reference's benchmark does (benchmark.jl:49)."""
    from oracle import matgen
    from oracle import rbl_oracle as o
    try:
        from threadpoolctl import threadpool_info, threadpool_limits
        threads = max([d.get("num_threads", 1) for d in threadpool_info()] or [1])
    except Exception:
        threadpool_limits = None
        threads = 1
    ns = min(args.cpu_sample_n, args.n)
    if args.matrix == "rmat":  # same draw density per row, ids scaled down with n
        sc = max(1, int(math.ceil(math.log2(ns))))
        A = matgen.rmat_csr(ns, sc, int(args.rmat_edges * ns / args.n), args.seed, plant)
    elif args.matrix == "circuit":
        A = matgen.circuit_like_csr(ns, args.seed, plant)
    else:
        A = matgen.hashwindow_csr(ns, args.halfwidth, args.density, args.seed, plant)
    omega = np.random.default_rng(0).standard_normal((ns, args.b))

    def timed():
        t0 = time.perf_counter()
        if args.basis_bits == 32:  # RBL_gpu.jl with FLOAT = Float32
            o.RBL_gpu_mixed(A, args.k, args.b, omega=omega, kryl_sz=args.kryl, check=False)
        else:
            o.RBL_gpu_semantics(A, args.k, args.b, omega=omega, kryl_sz=args.kryl, check=False)
        return time.perf_counter() - t0

    t = timed()
    scale = args.n / ns
    out = {"value": round(m_max / (t * scale), 5), "unit": "block iterations/s",
           "cores": threads, "kind": "port",
           "threads_note": f"{threads} BLAS threads of the box's {os.cpu_count()} CPUs: the harness's "
                           "OMP_NUM_THREADS for one GPU's share of the host",
           "sample": f"oracle RBL (RBL.jl restated, NumPy/SciPy OpenBLAS on {threads} threads; SpMM "
                     f"single-threaded as SparseArrays) on the same generator at n={ns} "
                     f"(nnz={A.nnz}) for the same {m_max} block steps: {t:.2f} s measured, i.e. "
                     f"{m_max / t:.4f} iters/s at n={ns}; value = that per-iteration time scaled "
                     f"x{scale:.0f} to n={args.n}",
           "sample_n": ns, "sample_seconds": round(t, 3),
           "sample_iters_per_s": round(m_max / t, 5),
           "host_cpus": os.cpu_count(), "cpu_model": cpu_model()}
    if not args.no_cpu_one_thread and threadpool_limits is not None:
        with threadpool_limits(limits=1):
            t1 = timed()
        out.update({"value_1thread": round(m_max / (t1 * scale), 5),
                    "sample_seconds_1thread": round(t1, 3)})
    if args.cpu_check_n and args.matrix == "hashwindow" and args.basis_bits == 64:
        out["linear_scaling_check"] = cpu_scaling_check(args, plant, A, omega)
    fixed_n = args.n if args.cpu_fixed_n < 0 else args.cpu_fixed_n
    if fixed_n and args.matrix == "hashwindow" and args.basis_bits == 64:
        # ~3.5 minutes at n = 1e7 (the 1e9-nnz CSR build + 8 oracle steps): by default only while
        # the run is young enough to finish well inside a 10-minute budget
        elapsed = time.perf_counter() - T_START
        if args.cpu_fixed_n < 0 and elapsed > CPU_FIXED_START_BY_S:
            out["fixed_steps_at_n"] = {"n": fixed_n, "skipped": f"the run was {elapsed:.0f} s old "
                                       f"(> {CPU_FIXED_START_BY_S} s); --cpu-fixed-n {fixed_n} forces it"}
        else:
            out["fixed_steps_at_n"] = cpu_fixed_steps(args, plant, fixed_n)
    out["value_is"] = ("the 38-step rate extrapolated linearly from the n = %d sample (sample, "
                       "linear_scaling_check); fixed_steps_at_n is SURVEY §8(d)'s fixed-step form "
                       "measured at the config's own n (the first steps only: the partial reorth "
                       "grows with the step, so it is not the 38-step rate)" % ns)
    return out


def cpu_fixed_steps(args, plant, n):
    """the oracle at the config's own n for a fixed number of block steps (rbl_start
    + the first --cpu-check-steps steps, convergence checks off), per-step time stated as such —
    not extrapolated.  The partial reorth grows with the step, so a 38-step run costs more per
    step than these first steps."""
    import threading
    from oracle import matgen
    from oracle import rbl_oracle as o
    steps = args.cpu_check_steps
    done = threading.Event()

    def heartbeat():  # minutes of CPU work: keep stderr alive
        while not done.wait(30.0):
            progress(f"CPU fixed-step run at n={n} in progress")
    hb = threading.Thread(target=heartbeat, daemon=True)
    hb.start()
    try:
        t0 = time.perf_counter()
        A = matgen.hashwindow_csr_chunked(n, args.halfwidth, args.density, args.seed, plant)
        gen_s = time.perf_counter() - t0
        progress(f"CPU fixed-step run: matrix built ({gen_s:.0f} s)")
        omega = np.random.default_rng(0).standard_normal((n, args.b))
        t0 = time.perf_counter()
        o.RBL_gpu_semantics(A, args.k, args.b, omega=omega, kryl_sz=args.kryl, check=False,
                            max_steps=steps)
        t = time.perf_counter() - t0
    finally:
        done.set()
    return {"n": n, "nnz": int(A.nnz), "block_steps": steps, "seconds": round(t, 2),
            "ms_per_block_step": round(t / steps * 1e3, 1),
            "block_iters_per_s_first_steps": round(steps / t, 5),
            "matrix_build_s": round(gen_s, 1),
            "note": "the oracle's rbl_start + first block steps at this n, measured in this run; the "
                    "38-step figure (`value`) is extrapolated from the n = 1e5 sample"}


def cpu_scaling_check(args, plant, A_small, omega_small):
    """Measured in this run: the first `--cpu-check-steps` block steps (a fixed-step run, SURVEY
    §8(d)) at the sample's n and at `--cpu-check-n` (10x by default), so the line itself shows
    how the per-step time grows with n — the basis of the sample's linear scaling to n = 1e7."""
    from oracle import matgen
    from oracle import rbl_oracle as o
    steps, n_big = args.cpu_check_steps, min(args.cpu_check_n, args.n)
    A_big = matgen.hashwindow_csr(n_big, args.halfwidth, args.density, args.seed, plant)
    omega_big = np.random.default_rng(0).standard_normal((n_big, args.b))

    def fixed(A, om):
        t0 = time.perf_counter()
        o.RBL_gpu_semantics(A, args.k, args.b, omega=om, kryl_sz=args.kryl, check=False,
                            max_steps=steps)
        return time.perf_counter() - t0

    t_small, t_big = fixed(A_small, omega_small), fixed(A_big, omega_big)
    n_small = A_small.shape[0]
    return {"block_steps": steps, "n_small": n_small, "seconds_small": round(t_small, 3),
            "n_big": n_big, "nnz_big": int(A_big.nnz), "seconds_big": round(t_big, 3),
            "time_ratio": round(t_big / t_small, 3), "n_ratio": round(n_big / n_small, 3),
            "ms_per_block_step_big": round(t_big / steps * 1e3, 1),
            "note": "rbl_start + the first block steps, convergence checks off, both timed in "
                    "this run on the same threads; time_ratio ~ n_ratio supports the linear "
                    "scaling of `value`"}


if __name__ == "__main__":
    main()
