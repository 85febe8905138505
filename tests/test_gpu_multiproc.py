"""GPU: the process-per-rank path with REAL processes on one GPU.

Every rank is its own process with its own HIP context (tests/mp_rank.py, started by
tests/rank_launcher.py), and the collectives go through the shared-memory transport
(rbl_create_shm) — the production orchestration of `bench.py --gpus N` with only RCCL swapped
out (RCCL refuses two ranks on one device).  Covered: the shm rendezvous, rbl_create_shm, the
setup collectives of every matrix kind (the nnz-balanced R-MAT split, the collective banded
vote, build_ghosts' request exchange), the indexed halo with the side-stream overlap, the range
halo a ghost-built context falls back to for b outside {16, 32} or a pinned gather kernel, fp64
and fp32 bases, and matrices replaced in place on one context (bench.py's sub-records).

The same cases also run over RCCL itself with 2, 3, 4 and 8 processes on the one GPU (8: the
largest point of the driver's 1 -> 8 curve; 3: a ragged, non-power-of-two split)
(tests/rccl_rank.py: each rank declares its own host id, so RCCL connects the ranks through its
network transport on the loopback interface instead of refusing two ranks on one device).

Checks, per world size 2 and 4:
  * every rank returns the same A_i / B_{i+1} bit for bit (the sums are formed identically);
  * bit for bit the in-process LocalComm run at the same P (threads in one process: the same
    partition, kernels and rank-order sums — so the process boundary changes nothing);
  * the single-rank run within 1e-10 relative per step (fp64; 1e-5 for the fp32 basis) —
    the partitioned sums only reorder additions;
  * the push/pull split of the indexed halo (RBL_OPT_HALO_PUSH 1, with and without the side
    stream) and the pull-all halo (0): the moved-row counts its setup predicted are the rows
    the exchanges moved;
  * BASELINE config 4 (R-MAT, n = 1e6) and config 3's shape against the oracle fixtures
    golden_c4b / golden_c3: same step count, eigenvalues < 1e-10.
"""
import os
import sys
import time
import uuid

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import mp_rank  # noqa: E402

pytestmark = pytest.mark.gpu

RM = {"matrix": "rmat", "n": 60000, "scale": 16, "edges": 60000 * 66, "seed": 7}
CASES = [
    {"name": "hw", "matrix": "hashwindow", "n": 9000, "W": 64, "p": 0.7734, "seed": 41, "b": 32,
     "steps": 10},
    {"name": "hw32", "matrix": "hashwindow", "n": 9000, "W": 64, "p": 0.7734, "seed": 41, "b": 32,
     "steps": 10, "bits": 32},
    # a wide band (half-width 600): the column panels over the range halo (kernel 7)
    {"name": "wide", "matrix": "hashwindow", "n": 40000, "W": 600, "p": 0.08, "seed": 43, "b": 32,
     "steps": 8, "kid": 7},
    {"name": "rmat", **RM, "b": 32, "steps": 10},                    # indexed halo + overlap
    {"name": "rmat_seq", **RM, "b": 32, "steps": 10, "overlap": 0},  # exchange before the SpMM
    {"name": "rmat_pull", **RM, "b": 32, "steps": 10, "push": 0},     # pull-all indexed halo
    {"name": "rmat_push", **RM, "b": 32, "steps": 10, "push": 1},     # push/pull split
    {"name": "rmat_push_seq", **RM, "b": 16, "steps": 10, "push": 1, "overlap": 0},
    {"name": "rmat32", **RM, "b": 32, "steps": 10, "bits": 32},
    {"name": "rmat_b8", **RM, "b": 8, "steps": 8},                    # range halo, ghost-built
    {"name": "rmat_gather", **RM, "b": 32, "steps": 6, "spmm_kernel": 1},
    {"name": "circ", "matrix": "circuit", "n": 20000, "width": 141, "seed": 5, "b": 16,
     "steps": 10},
    {"name": "c4b", "golden": "c4b", "b": 32},
    {"name": "c3", "golden": "c3", "b": 16},
]
TRACE_CASES = [c for c in CASES if not c.get("golden")]


@pytest.fixture(scope="module")
def rbl():
    import rbl as _r
    return _r


def _launch(rank_launcher, P, tmp):
    import json
    path = f"/dev/shm/rbl_test_{os.getpid()}_{uuid.uuid4().hex[:12]}"
    outs = [os.path.join(tmp, f"rank{r}.npz") for r in range(P)]
    cmds = [[sys.executable, "-u", os.path.join(HERE, "mp_rank.py"), "--path", path,
             "--nranks", str(P), "--rank", str(r), "--cases", json.dumps(CASES), "--out", outs[r]]
            for r in range(P)]
    t0 = time.time()
    rcs, logs = rank_launcher.run(cmds, timeout=300, env={"RBL_SHM_TIMEOUT_S": "60"})
    assert rcs == [0] * P, "\n".join(f"--- rank {r} rc={rc}\n{log}" for r, (rc, log) in
                                      enumerate(zip(rcs, logs)))
    assert not os.path.exists(path), "the shm segment outlived the group"
    print(f"P={P}: {time.time() - t0:.1f} s for {len(CASES)} cases")
    res = []
    for o in outs:
        with np.load(o) as z:
            res.append({k: z[k] for k in z.files})
    return res


@pytest.fixture(scope="module", params=[2, 4])
def procs(request, rank_launcher, tmp_path_factory):
    P = request.param
    return P, _launch(rank_launcher, P, str(tmp_path_factory.mktemp(f"mp{P}")))


@pytest.fixture(scope="module")
def single(rbl):
    out = {}
    with rbl.Context(0) as ctx:
        for c in TRACE_CASES:
            out[c["name"]] = mp_rank.run_case(rbl, ctx, c)
    return out


@pytest.fixture(scope="module")
def inproc(rbl):
    from test_gpu_multirank import run_ranks
    cache = {}

    def get(P):
        if P not in cache:
            def fn(ctx, r):
                return {c["name"]: mp_rank.run_case(rbl, ctx, c) for c in TRACE_CASES}
            cache[P] = run_ranks(rbl, P, fn, timeout=280)
        return cache[P]
    return get


def _launch_rccl(rank_launcher, P, tmp):
    """P processes of tests/rccl_rank.py, all on GPU 0, over RCCL itself (one host id per rank:
    RCCL's network transport on the loopback interface instead of xGMI)."""
    import json
    uid = os.path.join(tmp, "rccl_uid")
    outs = [os.path.join(tmp, f"rccl{r}.npz") for r in range(P)]
    cmds = [[sys.executable, "-u", os.path.join(HERE, "rccl_rank.py"), "--uid-file", uid,
             "--nranks", str(P), "--rank", str(r), "--cases", json.dumps(CASES), "--out", outs[r]]
            for r in range(P)]
    t0 = time.time()
    rcs, logs = rank_launcher.run(cmds, timeout=400, env={"NCCL_SOCKET_IFNAME": "lo",
                                                          "NCCL_DEBUG": "WARN"})
    assert rcs == [0] * P, "\n".join(f"--- rank {r} rc={rc}\n{log}" for r, (rc, log) in
                                      enumerate(zip(rcs, logs)))
    print(f"RCCL P={P}: {time.time() - t0:.1f} s for {len(CASES)} cases")
    res = []
    for o in outs:
        with np.load(o) as z:
            res.append({k: z[k] for k in z.files})
    return res


@pytest.fixture(scope="module", params=[2, 3, 4, 8])
def rccl_procs(request, rank_launcher, tmp_path_factory):
    P = request.param
    return P, _launch_rccl(rank_launcher, P, str(tmp_path_factory.mktemp(f"rccl{P}")))


@pytest.mark.parametrize("case", [c["name"] for c in TRACE_CASES])
def test_rccl_ranks_on_one_gpu(rccl_procs, single, inproc, case):
    """The production transport, RCCL (rbl_create_dist: ncclAllReduce, grouped ncclSend /
    ncclRecv, ncclAllGather in the setup), with real processes: every rank returns the same
    A_i / B_{i+1}; at 2 ranks bit for bit the in-process run (a two-term sum is the same in any
    order), at 4 within 1e-10 of the single-rank run like the other transports."""
    P, res = rccl_procs
    c = next(x for x in CASES if x["name"] == case)
    for r in res:
        assert str(r["transport"]) == "rccl" and int(r["transport_ranks"]) == P
    A0, B0 = res[0][f"{case}__A"], res[0][f"{case}__B"]
    assert len(A0) == c["steps"]
    for r in res[1:]:
        assert np.array_equal(r[f"{case}__A"], A0) and np.array_equal(r[f"{case}__B"], B0)
    if P == 2:
        ip = inproc(P)
        assert np.array_equal(ip[0][case]["A"], A0) and np.array_equal(ip[0][case]["B"], B0)
    tol = 1e-10 if c.get("bits", 64) == 64 else 1e-5
    s = single[case]
    for a, a1 in zip(list(A0) + list(B0), list(s["A"]) + list(s["B"])):
        assert np.abs(a - a1).max() <= tol * np.abs(a1).max()
    comm = [r[f"{case}__comm"] for r in res]
    assert all(cm[2] > 0 for cm in comm), "no halo exchange"
    if c.get("kid") is not None:
        assert all(int(r[f"{case}__kid"]) == c["kid"] for r in res), case
    if c.get("push") is not None:
        assert all(cm[2] == (c["steps"] + 1) * (2 if c["push"] else 1) for cm in comm)


def test_rccl_library_is_rocms(rccl_procs, rbl):
    """Every rank's RCCL transport calls ROCm's own RCCL (rbl_rccl_version: opened by path with
    a private symbol scope), the same copy as this process and as bench.py — whatever else a
    process loaded first (torch bundles another RCCL under the same soname)."""
    P, res = rccl_procs
    mine = rbl.rccl_version()
    print(f"RCCL P={P}: {mine}")
    assert mine["rccl_path"].startswith("/opt/rocm")
    for r in res:
        assert str(r["rccl_version"]) == mine["rccl_version"]
        assert str(r["rccl_path"]) == mine["rccl_path"]


@pytest.mark.parametrize("case", ["c4b", "c3"])
def test_rccl_golden_fixtures(rccl_procs, case):
    """BASELINE config 4 (R-MAT, n = 1e6, the push/pull split) and config 3's shape over RCCL
    on 2 and 4 processes: the oracle fixture's step count and eigenvalues (< 1e-10)."""
    P, res = rccl_procs
    g = np.load(os.path.join(HERE, "golden", f"golden_{case}.npz"))
    for r in res:
        assert bool(r[f"{case}__converged"]) and int(r[f"{case}__iters"]) == int(g["iters"])
        rel = np.abs(r[f"{case}__D"] - g["D"]) / np.abs(g["D"])
        assert rel.max() < 1e-10, rel


def test_transport_is_shm_processes(procs):
    P, res = procs
    for r in res:
        assert str(r["transport"]) == "shm" and int(r["transport_ranks"]) == P
    # the row slices tile [0, n) in rank order
    for c in CASES:
        r0 = [int(r[f"{c['name']}__r0"]) for r in res]
        r1 = [int(r[f"{c['name']}__r1"]) for r in res]
        assert r0[0] == 0 and r0[1:] == r1[:-1]


@pytest.mark.parametrize("case", [c["name"] for c in TRACE_CASES])
def test_ranks_agree_and_match_inprocess_and_single(procs, single, inproc, case):
    P, res = procs
    c = next(x for x in CASES if x["name"] == case)
    A0, B0 = res[0][f"{case}__A"], res[0][f"{case}__B"]
    assert len(A0) == c["steps"]
    for r in res[1:]:
        assert np.array_equal(r[f"{case}__A"], A0) and np.array_equal(r[f"{case}__B"], B0)
    # the same ranks as threads of one process (LocalComm): bit for bit
    ip = inproc(P)
    assert np.array_equal(ip[0][case]["A"], A0) and np.array_equal(ip[0][case]["B"], B0)
    # the single-rank run: the partitioned sums reorder additions only
    tol = 1e-10 if c.get("bits", 64) == 64 else 1e-5
    s = single[case]
    for a, a1 in zip(list(A0) + list(B0), list(s["A"]) + list(s["B"])):
        assert np.abs(a - a1).max() <= tol * np.abs(a1).max()
    # the kernels and exchanges the case is about really ran
    kid = int(res[0][f"{case}__kid"])
    comm = [r[f"{case}__comm"] for r in res]
    assert all(cm[2] > 0 for cm in comm), "no halo exchange"
    if c["matrix"] == "rmat" and c["b"] in (16, 32) and not c.get("spmm_kernel"):
        assert kid == 6  # segmented gather with the indexed halo
    if case in ("rmat_b8", "rmat_gather"):
        assert kid == 1  # plain gather over the range halo of a ghost-built context
    if c.get("kid") is not None:
        assert all(int(r[f"{case}__kid"]) == c["kid"] for r in res), case
    if c.get("push") is not None:  # the halo plan asked for, with its moved-row count exact
        for cm in comm:
            assert cm[5] == c["push"]
        rows = sum(int(cm[4]) for cm in comm) // ((c["steps"] + 1) * c["b"] * 8)
        assert rows == int(comm[0][6 if c["push"] else 7])
        assert all(cm[2] == (c["steps"] + 1) * (2 if c["push"] else 1) for cm in comm)


@pytest.mark.parametrize("case", ["c4b", "c3"])
def test_golden_fixtures_on_processes(procs, case):
    """BASELINE config 4 (R-MAT, n = 1e6, b = 32; the push/pull halo split on) and config 3's
    shape (n = 1,585,478, b = 16) on P processes: the oracle fixture's step count and eigenvalues
    (< 1e-10), Ritz rows
    gathered from the ranks matching the fixture's largest entries (1e-6, up to sign)."""
    P, res = procs
    g = np.load(os.path.join(HERE, "golden", f"golden_{case}.npz"))
    if case == "c4b":  # R-MAT's hubs: the automatic halo plan takes the push/pull split
        assert all(int(r["c4b__comm"][5]) == 1 for r in res)
    for r in res:
        assert bool(r[f"{case}__converged"]) and int(r[f"{case}__iters"]) == int(g["iters"])
        rel = np.abs(r[f"{case}__D"] - g["D"]) / np.abs(g["D"])
        assert rel.max() < 1e-10, rel
    V = np.vstack([r[f"{case}__V"] for r in res])
    idx, val = g["top_idx"], g["top_val"]
    for j in range(V.shape[1]):
        v = V[idx[:, j], j]
        sgn = np.sign(v @ val[:, j])
        assert np.abs(sgn * v - val[:, j]).max() < 1e-6
