#!/bin/bash
# round 6, batch 3: the column-panel SpMM's tests, then the half-width sweep (C4a-sized runs).
set -u
mkdir -p gpurun_out/r06_b3
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_multirank.py -m gpu -x -v \
  --timeout 200 --timeout-method thread -k "panel" > gpurun_out/r06_b3/pytest.log 2>&1; rc=$?
tail -15 gpurun_out/r06_b3/pytest.log
[ $rc -ne 0 ] && exit $rc
bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b3/hw
