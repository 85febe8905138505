#!/bin/bash
# round 6, batch 32: column panels with 6 rows per group (R = 384: <6, 16>, <6, 32>; probe builds
# tools/variants/p616, p632) against the product (v10: <4, 48> / <8, 16>) at H = 512 .. 2048;
# the panel tests on both variants first.
set -u
mkdir -p gpurun_out/r06_b32
export TMPDIR=/tmp
for v in p616 p632; do
  RBL_LIB=tools/variants/$v/librbl_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_multirank.py \
    -m gpu -x -q --timeout 200 --timeout-method thread -k "panel" > gpurun_out/r06_b32/pytest_$v.log 2>&1; rc=$?
  echo "$v: $(tail -1 gpurun_out/r06_b32/pytest_$v.log)"
  [ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06_b32/pytest_$v.log | head; exit $rc; }
done
for rep in 1 2; do
  echo "== product, rep $rep"
  bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b32/p$rep 512 768 1024 2048 || exit 1
  for v in p616 p632; do
    echo "== $v, rep $rep"
    RBL_LIB=tools/variants/$v/librbl_hip.so bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b32/$v$rep 512 768 1024 2048 || exit 1
  done
done
