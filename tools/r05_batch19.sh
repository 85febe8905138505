#!/bin/bash
# round 5, batch 19: the N = 8 RCCL rehearsal of the whole default job on the final tree (8
# processes sharing the one GPU, each its own RCCL host over loopback; progress on stderr)
set -u
mkdir -p gpurun_out/r05_b19
export TMPDIR=/tmp
RBL_RCCL_HOST_PER_RANK=1 NCCL_DEBUG=WARN timeout -k 20 900 python bench.py --gpus 8 --n 2000000 \
  --steps 2 --warmup 1 --rmat-steps 1 --rmat-as-drawn-steps 0 --c3-steps 1 --no-ttk-slow \
  --c5-n 8000000 --c5-steps 1 > gpurun_out/r05_b19/rccl8.json 2> gpurun_out/r05_b19/rccl8.err; rc=$?
echo "rccl8 bench rc=$rc"; grep "^\[bench" gpurun_out/r05_b19/rccl8.err | tail -3
python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b19/rccl8.json').read().strip().splitlines()[-1])
print(d['value'], d['comm_per_step'], d['config'].get('rccl_version'))
for k in ('c4b_rmat','c3_circuit','c5'):
    r=d.get(k) or {}; print(k, r.get('value'), r.get('comm_per_step'))"
exit $rc
