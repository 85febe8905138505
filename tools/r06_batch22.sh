#!/bin/bash
# round 6, batch 22: column-panel v8 (early Q_{i-1} loads for <4,32>, epilogue loads batched,
# unconditional record prefetch) — tests and the sweep.
set -u
mkdir -p gpurun_out/r06_b22
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_multirank.py tests/test_gpu_parity.py \
  -m gpu -x -v --timeout 200 --timeout-method thread -k "panel or c1" > gpurun_out/r06_b22/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06_b22/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06_b22/pytest.log | head; exit $rc; }
bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b22/hw 128 256 512 1024 2048 || exit 1
