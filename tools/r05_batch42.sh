#!/bin/bash
# round 5, batch 42: probe — a one-wave kernel kept resident on a side stream for 60 ms after each
# rbl_fetch (RBL_KEEPALIVE_MS), so the GPU is not idle during the host eigensolve: does the slow
# run's first-Ritz wait (11-32 ms in bench.py's order) go away?
set -u
mkdir -p gpurun_out/r05_b42
export TMPDIR=/tmp
for v in 60 none 60 none; do
  unset RBL_KEEPALIVE_MS; [ $v != none ] && export RBL_KEEPALIVE_MS=$v
  echo "== keepalive $v" >> gpurun_out/r05_b42/p.log
  RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ritz_sync_probe.py bench >> gpurun_out/r05_b42/p.log 2>&1 || { cat gpurun_out/r05_b42/p.log; exit 1; }
done
cat gpurun_out/r05_b42/p.log
