#!/bin/bash
# round 5, batch 38: does a stream sync in rbl_fetch (instead of the step's event) take the
# ~20 ms that the slow run's first rbl_ritz waits on an idle stream?
set -u
mkdir -p gpurun_out/r05_b38
export TMPDIR=/tmp
for f in 1 0; do
  if [ $f = 1 ]; then export RBL_FETCH_STREAMSYNC=1; else unset RBL_FETCH_STREAMSYNC; fi
  echo "== RBL_FETCH_STREAMSYNC=$f" >> gpurun_out/r05_b38/p.log
  RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ritz_sync_probe.py bench >> gpurun_out/r05_b38/p.log 2>&1 || { cat gpurun_out/r05_b38/p.log; exit 1; }
done
cat gpurun_out/r05_b38/p.log | grep -v "stream sync at step [0-9] \|stream sync at step 1[0-9] "
