#!/bin/bash
# round 5, batch 30: same-box A/B of the bench's time-to-k with and without the residual-driven
# speculation (3 alternating pairs, sub-records and CPU baseline off), then the default line.
set -u
mkdir -p gpurun_out/r05_b30
export TMPDIR=/tmp
for rep in 1 2 3; do
  for sp in off auto; do
    timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --rmat-steps 0 --c3-steps 0 \
      --speculate $sp > gpurun_out/r05_b30/ab_${sp}_$rep.json 2> gpurun_out/r05_b30/ab_${sp}_$rep.err || { tail -5 gpurun_out/r05_b30/ab_${sp}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b30/ab_${sp}_$rep.json').read().strip().splitlines()[-1])
t=d['time_to_k']; s=d['time_to_k_slow_spectrum']
print('$sp', $rep, 'planted', t['seconds'], t['host_ms'], 'slow', s['seconds'], s['host_ms'], s['speculated_steps'], s['speculated_discarded'])" | tee -a gpurun_out/r05_b30/ab.log
  done
done
timeout -k 10 600 python bench.py > gpurun_out/r05_b30/bench.json 2> gpurun_out/r05_b30/bench.err || { tail -5 gpurun_out/r05_b30/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b30/bench.json').read().strip().splitlines()[-1])
print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_secondary']['frac'])
t=d['time_to_k']; s=d['time_to_k_slow_spectrum']
print('ttk', t['seconds'], t['host_ms'], 'slow', s['seconds'], s['host_ms'], s['speculated_steps'], s['speculated_discarded'])
print('c4b', d['c4b_rmat']['value'], 'c3', d['c3_circuit']['value'])"
