#!/bin/bash
# round 5, batch 39: is the ~20 ms stall of the slow run's first rbl_ritz copy the copy engine
# waking?  bench-order probe: default, S uploaded by a kernel from mapped memory, a tiny D2H per fetch.
set -u
mkdir -p gpurun_out/r05_b39
export TMPDIR=/tmp
for v in none skernel warm none skernel warm; do
  unset RBL_RITZ_S_KERNEL RBL_FETCH_WARM
  [ $v = skernel ] && export RBL_RITZ_S_KERNEL=1
  [ $v = warm ] && export RBL_FETCH_WARM=1
  echo "== $v" >> gpurun_out/r05_b39/p.log
  RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ritz_sync_probe.py bench >> gpurun_out/r05_b39/p.log 2>&1 || { cat gpurun_out/r05_b39/p.log; exit 1; }
done
grep -v "stream idle at entry after 0\.\|^rbl_ritz: S rows + H2D done at 0\." gpurun_out/r05_b39/p.log
