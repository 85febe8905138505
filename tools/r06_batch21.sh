#!/bin/bash
# round 6, batch 21: column-panel v7 (the wave's largest count per row from two ds_bpermute
# maxima per step instead of four readlanes per row) — tests and the sweep; then the same-box
# A/B of the C4a line against the round-5 final tree (tools/r06_batch20.sh).
set -u
mkdir -p gpurun_out/r06_b21
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_multirank.py tests/test_gpu_parity.py \
  -m gpu -x -v --timeout 200 --timeout-method thread -k "panel or c1" > gpurun_out/r06_b21/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06_b21/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06_b21/pytest.log | head; exit $rc; }
bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b21/hw 128 256 512 1024 2048 || exit 1
bash tools/r06_batch20.sh || exit 1
