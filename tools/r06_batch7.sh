#!/bin/bash
# round 6, batch 7: column-panel SpMM v3 (exact counts, buffer loads, 512-row blocks) — tests, the
# half-width sweep, and the same sweep with the segmented gather forced (the kernel the
# library chose for these bands before the column panels).
set -u
mkdir -p gpurun_out/r06_b7
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_multirank.py -m gpu -x -v \
  --timeout 200 --timeout-method thread -k "panel" > gpurun_out/r06_b7/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06_b7/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06_b7/pytest.log | head; exit $rc; }
bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b7/hw 128 256 512 1024 2048 || exit 1

