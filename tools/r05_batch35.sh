#!/bin/bash
# round 5, batch 35: the Ritz coefficient upload through the pinned staging slot vs from pageable
# memory (RBL_RITZ_PAGEABLE_S=1), inside bench.py's time-to-k runs, alternating.
set -u
mkdir -p gpurun_out/r05_b35
export TMPDIR=/tmp
for rep in 1 2; do
  for pg in 1 0; do
    if [ $pg = 1 ]; then export RBL_RITZ_PAGEABLE_S=1; else unset RBL_RITZ_PAGEABLE_S; fi
    RBL_RITZ_TRACE=1 timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --rmat-steps 0 --c3-steps 0 \
      > gpurun_out/r05_b35/ab_${pg}_$rep.json 2> gpurun_out/r05_b35/ab_${pg}_$rep.err || { tail -5 gpurun_out/r05_b35/ab_${pg}_$rep.err; exit 1; }
    echo "== pageable_S=$pg rep $rep" >> gpurun_out/r05_b35/ab.log
    grep rbl_ritz gpurun_out/r05_b35/ab_${pg}_$rep.err >> gpurun_out/r05_b35/ab.log
    python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b35/ab_${pg}_$rep.json').read().strip().splitlines()[-1])
t=d['time_to_k']; s=d['time_to_k_slow_spectrum']
print('planted', t['seconds'], t['host_ms'], 'slow', s['seconds'], s['host_ms'])" >> gpurun_out/r05_b35/ab.log
  done
done
cat gpurun_out/r05_b35/ab.log
