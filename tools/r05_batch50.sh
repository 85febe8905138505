#!/bin/bash
# round 5, batch 50: the 2-step speculation tier (pred in (5 tol, 100 tol]) vs without it
# (RBL_SPEC_MID=0): the slow-spectrum time-to-k probe and the bench's time-to-k, alternating.
set -u
mkdir -p gpurun_out/r05_b50
export TMPDIR=/tmp
for mid in 0 1 0 1; do
  echo "== RBL_SPEC_MID=$mid" >> gpurun_out/r05_b50/ttk.log
  RBL_SPEC_MID=$mid timeout -k 10 200 python -u tools/r05_ttk_probe.py slow >> gpurun_out/r05_b50/ttk.log 2>&1 || { cat gpurun_out/r05_b50/ttk.log; exit 1; }
done
cat gpurun_out/r05_b50/ttk.log
for rep in 1 2; do
  for mid in 0 1; do
    RBL_SPEC_MID=$mid timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --rmat-steps 0 --c3-steps 0 \
      > gpurun_out/r05_b50/ab_${mid}_$rep.json 2> gpurun_out/r05_b50/ab_${mid}_$rep.err || { tail -5 gpurun_out/r05_b50/ab_${mid}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b50/ab_${mid}_$rep.json').read().strip().splitlines()[-1])
t=d['time_to_k']; s=d['time_to_k_slow_spectrum']
print('mid=$mid', $rep, 'planted', t['seconds'], 'slow', s['seconds'], s['host_ms'], s['speculated_steps'], s['speculated_discarded'])" | tee -a gpurun_out/r05_b50/ab.log
  done
done
