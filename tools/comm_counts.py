#!/usr/bin/env python3
"""Collectives per block step at P in-process ranks (LocalGroup on one GPU): the counts and
bytes rbl_comm_stats reports for the bench's three patterns at a reduced n (the counts per step
do not depend on n; the halo bytes scale with n and are extrapolated to the bench's n below).
The R-MAT pattern runs three times: as drawn (hubs at the low ids) and relabelled (RBL_OPT_RELABEL,
the hubs spread over the row range), to show the sender balance the relabel buys, both with the
pull-all indexed halo; then relabelled with the push/pull split (RBL_OPT_HALO_PUSH 1), to show
the moved rows the split saves.
Usage: python tools/comm_counts.py [P] [tag]"""
import json
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gpu-randomized-block-lanczos_amd")]
import numpy as np  # noqa: E402
import rbl  # noqa: E402

from rbl import _lib  # noqa: E402

P = int(sys.argv[1]) if len(sys.argv) > 1 else 8
TAG = sys.argv[2] if len(sys.argv) > 2 else "r04"
plant = np.array([100.0 * (41 - l) for l in range(1, 41)])


def rmat(c, relabel, push):
    c.set_option(_lib.RBL_OPT_RELABEL, relabel)
    c.set_option(_lib.RBL_OPT_HALO_PUSH, push)
    c.gen_rmat(400_000, 19, int(0.66 * 100 * 400_000), 20261015, plant)
    c.set_option(_lib.RBL_OPT_RELABEL, 0)


cases = {
    "hashwindow (C4a pattern)": (lambda c: c.gen_hashwindow(400_000, 64, 0.7734, 20261015, plant), 32, 400_000, 10_000_000),
    "rmat (C4b pattern)": (lambda c: rmat(c, 0, 0), 32, 400_000, 10_000_000),
    "rmat relabelled (C4b pattern, RBL_OPT_RELABEL)": (lambda c: rmat(c, 1, 0), 32, 400_000, 10_000_000),
    "rmat relabelled, push/pull split (RBL_OPT_HALO_PUSH 1)": (lambda c: rmat(c, 1, 1), 32, 400_000, 10_000_000),
    "circuit (C3 shape)": (lambda c: c.gen_circuit(1_585_478, 20261015, plant), 16, 1_585_478, 1_585_478),
}
out = {}
for name, (gen, b, n, n_bench) in cases.items():
    steps = 38 if b == 32 else 75
    res = [None] * P
    group = rbl.LocalGroup(P)

    def worker(r):
        with rbl.Context(0, group=group, rank=r) as ctx:
            gen(ctx)
            ctx.comm_stats(reset=True)
            rbl.lanczos(ctx, 20, b, seed=3, check=False, ritz=False)
            res[r] = ctx.comm_stats()

    th = [threading.Thread(target=worker, args=(r,)) for r in range(P)]
    for t in th:
        t.start()
    for t in th:
        t.join(600)
    group.close()
    spmm = steps + 1
    plan_keys = ("halo_push", "push_rows_pred", "pull_rows_pred")
    per = {k: [round(s[k] / spmm, 2) for s in res] for k in res[0] if k not in plan_keys}
    scale = n_bench / n
    out[name] = {"P": P, "b": b, "n_measured": n, "block_steps": steps,
                 "per_spmm_step_by_rank": per,
                 "halo_plan": {k: res[0][k] for k in plan_keys},
                 "recv_bytes_per_step_max_rank_at_bench_n": max(per["recv_bytes"]) * scale,
                 "send_bytes_per_step_max_rank_at_bench_n": max(per["send_bytes"]) * scale,
                 "send_max_over_mean": max(per["send_bytes"]) / max(1e-9, sum(per["send_bytes"]) / P)}
    print(name, json.dumps(out[name]), flush=True)
json.dump(out, open(os.path.join(ROOT, "gpurun_out", f"{TAG}_comm_counts_P{P}.json"), "w"), indent=1)
