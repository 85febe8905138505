#!/bin/bash
# round 5, batch 37: which step of bench.py's time-to-k sequence makes the slow run's rbl_ritz wait
set -u
mkdir -p gpurun_out/r05_b37
export TMPDIR=/tmp
for v in bench noplant early fresh; do
  RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ritz_sync_probe.py $v >> gpurun_out/r05_b37/p.log 2>&1 || { cat gpurun_out/r05_b37/p.log; exit 1; }
done
cat gpurun_out/r05_b37/p.log
