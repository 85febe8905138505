#!/bin/bash
# round 5, batch 33: the bench's slow-spectrum Ritz + D2H (~70 ms against ~48 in the probe): the
# rbl_ritz host split inside bench.py (RBL_RITZ_TRACE), twice.
set -u
mkdir -p gpurun_out/r05_b33
export TMPDIR=/tmp
for rep in 1 2; do
  RBL_RITZ_TRACE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --rmat-steps 0 --c3-steps 0 \
    > gpurun_out/r05_b33/ab_$rep.json 2> gpurun_out/r05_b33/ab_$rep.err || { tail -5 gpurun_out/r05_b33/ab_$rep.err; exit 1; }
  grep rbl_ritz gpurun_out/r05_b33/ab_$rep.err
  python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b33/ab_$rep.json').read().strip().splitlines()[-1])
t=d['time_to_k']; s=d['time_to_k_slow_spectrum']
print($rep, 'planted', t['seconds'], t['host_ms'], 'slow', s['seconds'], s['host_ms'])"
done
