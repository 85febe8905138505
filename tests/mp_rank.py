"""One rank of a multi-process run over the shared-memory transport (rbl_create_shm): started
by tests/rank_launcher.py for tests/test_gpu_multiproc.py, one process per rank, all on GPU 0.

    python tests/mp_rank.py --path /dev/shm/rbl_x --nranks P --rank r --cases JSON --out f.npz

Runs every case of the JSON list on ONE context (each case generates its matrix in place of the
last, as bench.py's sub-records do) and saves, per case, the A_i / B_{i+1} traces, D, this rank's
Ritz rows, its row range, the SpMM kernel id and the collectives it issued.
"""
import argparse
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
for p in (ROOT, os.path.join(ROOT, "gpu-randomized-block-lanczos_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402


def planted(k):
    return np.array([100.0 * (2 * k + 1 - l) for l in range(1, 2 * k + 1)])


def golden_cfg(name):
    g = np.load(os.path.join(HERE, "golden", f"golden_{name}.npz"))
    return {k[4:]: g[k].item() for k in g.files if k.startswith("cfg_")}


def run_case(rbl, ctx, c):
    from rbl import _lib
    k, b = c.get("k", 10), c["b"]
    omega = None
    # read when the matrix is set: the push/pull split of the indexed halo (2: automatic)
    ctx.set_option(_lib.RBL_OPT_HALO_PUSH, c.get("push", 2))
    if c.get("golden"):
        cfg = golden_cfg(c["golden"])
        k, b = cfg["k"], cfg["b"]
        if c["golden"] == "c4b":
            ctx.gen_rmat(cfg["n"], cfg["scale"], cfg["edges"], cfg["seed"], planted(k))
        else:
            ctx.gen_circuit(cfg["n"], cfg["seed"], planted(k))
        n = cfg["n"]
        _, r0, r1, _ = ctx.matrix_info()
        omega = np.random.default_rng(cfg["omega_seed"]).standard_normal((n, b))[r0:r1]
    elif c["matrix"] == "hashwindow":
        ctx.gen_hashwindow(c["n"], c["W"], c["p"], c["seed"], planted(k))
    elif c["matrix"] == "rmat":
        ctx.gen_rmat(c["n"], c["scale"], c["edges"], c["seed"], planted(k))
    elif c["matrix"] == "circuit":
        ctx.gen_circuit(c["n"], c["seed"], planted(k), width=c["width"])
    else:
        raise ValueError(c)
    ctx.set_option(_lib.RBL_OPT_HALO_OVERLAP, c.get("overlap", 1))
    ctx.set_option(_lib.RBL_OPT_SPMM_KERNEL, c.get("spmm_kernel", 0))
    _, r0, r1, nnz = ctx.matrix_info()
    kid = ctx.spmm_kernel_for(b)
    ctx.comm_stats(reset=True)
    check = bool(c.get("golden")) or c.get("check", False)
    D, V, info = rbl.lanczos(ctx, k, b, omega=omega, seed=c.get("lseed", 3), check=check,
                             max_steps=None if check else c["steps"], trace=True, ritz=check,
                             basis_bits=c.get("bits", 64))
    comm = ctx.comm_stats()
    out = {"A": np.array(info.trace_A), "B": np.array(info.trace_B), "D": np.asarray(D),
           "iters": info.iters, "converged": info.converged, "r0": r0, "r1": r1, "nnz": nnz,
           "kid": kid, "comm": np.array([comm[x] for x in ("allreduce_calls", "allreduce_bytes",
                                                            "exchange_calls", "send_bytes",
                                                            "recv_bytes", "halo_push",
                                                            "push_rows_pred", "pull_rows_pred")])}
    if V is not None:
        out["V"] = V
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--path", required=True)
    ap.add_argument("--nranks", type=int, required=True)
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--cases", required=True)
    ap.add_argument("--out", required=True)
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args()
    import rbl
    cases = json.loads(a.cases)
    res = {}
    with rbl.Context(a.device, nranks=a.nranks, rank=a.rank, shm_path=a.path) as ctx:
        info = ctx.comm_info()
        res["transport"] = np.array(info["transport"])
        res["transport_ranks"] = info["nranks"]
        for c in cases:
            for key, v in run_case(rbl, ctx, c).items():
                res[f"{c['name']}__{key}"] = v
            print(f"rank {a.rank}: case {c['name']} done", flush=True)
    np.savez(a.out, **res)


if __name__ == "__main__":
    main()
