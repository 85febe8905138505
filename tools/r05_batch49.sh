#!/bin/bash
# round 5, batch 49: the bench-order first-Ritz wait with the planted V kept alive (no munmap of the
# 1.6 GB result just before the slow run) vs dropped
set -u
mkdir -p gpurun_out/r05_b49
export TMPDIR=/tmp
for v in keepv bench keepv bench; do
  RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ritz_sync_probe.py $v >> gpurun_out/r05_b49/p.log 2>&1 || { cat gpurun_out/r05_b49/p.log; exit 1; }
done
grep -v "^rbl_ritz" gpurun_out/r05_b49/p.log
