#!/bin/bash
# round 5, batch 40: residual-driven speculation across 8 RCCL processes (the driver's N = 8 time-to-k
# path): the default job at n = 2e6 with the slow-spectrum time-to-k on, beside one rank at the same n.
set -u
mkdir -p gpurun_out/r05_b40
export TMPDIR=/tmp
RBL_RCCL_HOST_PER_RANK=1 NCCL_DEBUG=WARN timeout -k 20 900 python bench.py --gpus 8 --n 2000000 \
  --steps 2 --warmup 1 --rmat-steps 1 --rmat-as-drawn-steps 0 --c3-steps 1 \
  --c5-n 8000000 --c5-steps 1 > gpurun_out/r05_b40/rccl8.json 2> gpurun_out/r05_b40/rccl8.err; rc=$?
echo "rccl8 bench rc=$rc"; grep "^\[bench" gpurun_out/r05_b40/rccl8.err | tail -3
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --n 2000000 --steps 2 --warmup 1 --no-cpu-baseline --rmat-steps 0 --c3-steps 0 \
  > gpurun_out/r05_b40/one.json 2> gpurun_out/r05_b40/one.err || { tail -5 gpurun_out/r05_b40/one.err; exit 1; }
python3 -c "
import json
for f in ('rccl8', 'one'):
    d=json.loads(open('gpurun_out/r05_b40/%s.json' % f).read().strip().splitlines()[-1])
    t=d['time_to_k']; s=d['time_to_k_slow_spectrum']
    print(f, d['n_gpus'], d['value'], d['config'].get('transport_ranks'), d['config'].get('rccl_version'))
    print('  planted', t['seconds'], t['iters'], t['top_eigenvalues'], t.get('speculated_steps'))
    print('  slow', s['seconds'], s['iters'], s['top_eigenvalues'], s['kth_eigenvalue'], s.get('speculated_steps'), s.get('speculated_discarded'), s.get('max_residual_per_check'))"
