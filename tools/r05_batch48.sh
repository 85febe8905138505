#!/bin/bash
# round 5, batch 48: the bench-order first-Ritz wait with the copy engines off (HSA_ENABLE_SDMA=0:
# copies as blit kernels) vs on — is the SDMA engine involved?
set -u
mkdir -p gpurun_out/r05_b48
export TMPDIR=/tmp
for v in 0 1 0 1; do
  echo "== HSA_ENABLE_SDMA=$v" >> gpurun_out/r05_b48/p.log
  HSA_ENABLE_SDMA=$v RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ritz_sync_probe.py bench >> gpurun_out/r05_b48/p.log 2>&1 || { cat gpurun_out/r05_b48/p.log; exit 1; }
done
cat gpurun_out/r05_b48/p.log
