"""One rank of a 2-process RCCL job with both ranks on GPU 0 (tests/test_gpu_multiproc.py).

RCCL refuses two ranks of one communicator on one device ("Duplicate GPU detected") when it
believes they share a host; each rank here declares its own host id (NCCL_HOSTID), so RCCL
connects them through its network transport over the loopback interface.  The collectives and
grouped send/recv the library issues are then the production RcclComm calls (rbl_create_dist,
ncclAllReduce / ncclAllGather / ncclSend / ncclRecv in groups), run for real; only the wire
differs from xGMI.

    python tests/rccl_rank.py --uid-file F --nranks P --rank r --cases JSON --out f.npz

Rank 0 writes the RCCL unique id to F; the others wait for it.  Per case, the same record as
tests/mp_rank.py (traces, D, Ritz rows, collectives).
"""
import argparse
import json
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import mp_rank  # noqa: E402  (sets sys.path for rbl)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--uid-file", required=True)
    ap.add_argument("--nranks", type=int, required=True)
    ap.add_argument("--rank", type=int, required=True)
    ap.add_argument("--cases", required=True)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    # read by RCCL when the communicator is created: one "host" per rank, loopback sockets
    os.environ["NCCL_HOSTID"] = f"rbl-test-host-{a.rank}"
    os.environ.setdefault("NCCL_SOCKET_IFNAME", "lo")
    import numpy as np
    import rbl
    from rbl import _lib
    if a.rank == 0:
        buf = np.zeros(128, np.uint8)
        st = _lib.lib.rbl_get_unique_id(_lib.u8ptr(buf))
        assert st == 0, "rbl_get_unique_id failed"
        tmp = a.uid_file + ".tmp"
        with open(tmp, "wb") as f:
            f.write(bytes(buf))
        os.replace(tmp, a.uid_file)
    t0 = time.time()
    while not os.path.exists(a.uid_file):
        if time.time() - t0 > 60:
            sys.exit("no unique id from rank 0")
        time.sleep(0.05)
    with open(a.uid_file, "rb") as f:
        uid = f.read()
    cases = json.loads(a.cases)
    res = {}
    with rbl.Context(0, nranks=a.nranks, rank=a.rank, unique_id=uid) as ctx:
        info = ctx.comm_info()
        res["transport"] = np.array(info["transport"])
        res["transport_ranks"] = info["nranks"]
        res["rccl_version"] = np.array(info["rccl_version"])
        res["rccl_path"] = np.array(info["rccl_path"])
        for c in cases:
            for key, v in mp_rank.run_case(rbl, ctx, c).items():
                res[f"{c['name']}__{key}"] = v
            print(f"rank {a.rank}: case {c['name']} done", flush=True)
    np.savez(a.out, **res)


if __name__ == "__main__":
    main()
