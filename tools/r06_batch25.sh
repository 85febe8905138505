#!/bin/bash
# round 6, batch 25: the final tree's whole default job (C4a with both time-to-k runs, C4b, C3,
# the wide band, C5 at n = 8e6) on 8 RCCL processes sharing the one GPU (one host id per rank,
# queues capped by bench.py) — every sub-record must complete on the N = 8 path.
set -u
mkdir -p gpurun_out/r06_b25
export TMPDIR=/tmp RBL_RCCL_HOST_PER_RANK=1
NCCL_DEBUG=WARN timeout -k 20 1000 python bench.py --gpus 8 --steps 2 --warmup 1 --c5-n 8000000 \
  --no-cpu-baseline > gpurun_out/r06_b25/rccl8.json 2> gpurun_out/r06_b25/rccl8.err; rc=$?
echo "rc=$rc"
[ $rc -ne 0 ] && { tail -30 gpurun_out/r06_b25/rccl8.err; exit $rc; }
python3 - gpurun_out/r06_b25/rccl8.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("C4a", d["value"], "ttk", d["time_to_k"]["seconds"], d["time_to_k_slow_spectrum"]["seconds"])
for k in ("c4b_rmat", "c3_circuit", "c4w_wideband", "c5_mixed"):
    x = d.get(k)
    print(k, None if x is None else (x.get("error") or (x.get("value"), (x.get("time_to_k") or {}).get("seconds"))))
PY
