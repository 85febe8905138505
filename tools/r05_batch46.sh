#!/bin/bash
# round 5, batch 46: the pipelined Ritz on 2 RCCL processes (n = 1e7: 5e6 rows per rank, so each
# rank's rbl_ritz takes the row-piece path) — the driver's N = 2 point rehearsed on one GPU.
set -u
mkdir -p gpurun_out/r05_b46
export TMPDIR=/tmp
RBL_RCCL_HOST_PER_RANK=1 NCCL_DEBUG=WARN RBL_RITZ_TRACE=1 timeout -k 20 900 python bench.py --gpus 2 \
  --steps 1 --warmup 1 --rmat-steps 1 --rmat-as-drawn-steps 0 --c3-steps 1 \
  --c5-n 8000000 --c5-steps 1 > gpurun_out/r05_b46/rccl2.json 2> gpurun_out/r05_b46/rccl2.err; rc=$?
echo "rccl2 bench rc=$rc"; grep "^\[bench" gpurun_out/r05_b46/rccl2.err | tail -2; grep "rbl_ritz" gpurun_out/r05_b46/rccl2.err | head -8
[ $rc -ne 0 ] && exit $rc
python3 -c "
import json
d=json.loads(open('gpurun_out/r05_b46/rccl2.json').read().strip().splitlines()[-1])
t=d['time_to_k']; s=d['time_to_k_slow_spectrum']
print(d['value'], d['config'].get('transport_ranks'), d['config'].get('rccl_version'))
print('planted', t['seconds'], t['iters'], t['top_eigenvalues'])
print('slow', s['seconds'], s['iters'], s['top_eigenvalues'], s['kth_eigenvalue'], s.get('speculated_steps'), s.get('max_residual_per_check'))
one=json.loads(open('profiles/r05_bench_b45_default.json').read().strip().splitlines()[-1])
print('one-rank planted', one['time_to_k']['top_eigenvalues'], 'slow', one['time_to_k_slow_spectrum']['top_eigenvalues'], one['time_to_k_slow_spectrum']['kth_eigenvalue'])"
