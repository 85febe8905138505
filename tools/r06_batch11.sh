#!/bin/bash
# round 6, batch 11: column-panel SpMM v4 (records regrouped panel-major, one-byte columns) —
# its tests and the R-MAT halo test the panel vote broke, then the half-width sweep.
set -u
mkdir -p gpurun_out/r06_b11
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_multirank.py tests/test_gpu_rmat.py \
  -m gpu -x -v --timeout 200 --timeout-method thread -k "panel or halo_overlap" > gpurun_out/r06_b11/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06_b11/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06_b11/pytest.log | head; exit $rc; }
bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b11/hw 128 256 512 1024 2048 || exit 1
