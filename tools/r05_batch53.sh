#!/bin/bash
# round 5, batch 53: the driver's N = 4 point at its own n (1e7: 2.5e6 rows per rank, so each rank's Ritz takes the row pieces) rehearsed as
# 4 RCCL processes on the one GPU, on the final tree (speculation, the Ritz side stream created at
# start) — C4a with both time-to-k runs, C4b, C3, and C5 at reduced n.
set -u
mkdir -p gpurun_out/r05_b53
export TMPDIR=/tmp
RBL_RCCL_HOST_PER_RANK=1 NCCL_DEBUG=WARN timeout -k 20 1000 python bench.py --gpus 4 \
  --steps 1 --warmup 1 --rmat-steps 1 --rmat-as-drawn-steps 0 --c3-steps 1 \
  --c5-n 8000000 --c5-steps 1 > gpurun_out/r05_b53/rccl4.json 2> gpurun_out/r05_b53/rccl4.err; rc=$?
echo "rccl4 bench rc=$rc"; grep "^\[bench" gpurun_out/r05_b53/rccl4.err | tail -3
[ $rc -ne 0 ] && { tail -20 gpurun_out/r05_b53/rccl4.err; exit $rc; }
python3 -c "
import json
d=json.loads(open('gpurun_out/r05_b53/rccl4.json').read().strip().splitlines()[-1])
t=d['time_to_k']; s=d['time_to_k_slow_spectrum']
print(d['value'], d['config'].get('transport_ranks'), d['config'].get('rccl_version'), d['comm_per_step'])
print('planted', t['seconds'], t['iters'], t['top_eigenvalues'])
print('slow', s['seconds'], s['iters'], s['top_eigenvalues'], s['kth_eigenvalue'], s.get('speculated_steps'), s.get('speculated_discarded'))
for k in ('c4b_rmat', 'c3_circuit', 'c5_mixed'):
    r = d.get(k) or {}; print(k, r.get('value'), (r.get('time_to_k') or {}).get('top_eigenvalues'), r.get('error'))"
