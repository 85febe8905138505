#!/bin/bash
# round 6, batch 24: residue-aligned panel order (product) against the ascending order
# (tools/variants/order0) — panel tests on the product, then alternating sweeps at H = 256, 1024.
set -u
mkdir -p gpurun_out/r06_b24
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_multirank.py \
  -m gpu -x -v --timeout 200 --timeout-method thread -k "panel" > gpurun_out/r06_b24/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06_b24/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06_b24/pytest.log | head; exit $rc; }
for rep in 1 2; do
  echo "== product (residue order), rep $rep"
  bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b24/res$rep 256 1024 2048 || exit 1
  echo "== order0 (ascending), rep $rep"
  RBL_LIB=tools/variants/order0/librbl_hip.so bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b24/asc$rep 256 1024 2048 || exit 1
done
