#!/bin/bash
# round 6, batch 31: the product with <4, 48> for rows with more than 16 entries per panel on
# average — panel tests, the wide-band full-size test, and the half-width sweep.
set -u
mkdir -p gpurun_out/r06_b31
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_multirank.py tests/test_gpu_wideband_fullsize.py \
  -m gpu -x -q --timeout 300 --timeout-method thread -k "panel or wideband" > gpurun_out/r06_b31/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06_b31/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06_b31/pytest.log | head; exit $rc; }
bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b31/hw 128 256 512 768 1024 2048
