#!/bin/bash
# round 6, batch 15: column-panel v5 (LDS reads one quad ahead of their FMAs, inline-asm reads
# with counted lgkmcnt) — its tests and the half-width sweep; then the P = 7 / 8 rehearsals with
# bench.py's cap (one hardware queue per process beyond 6 processes on a GPU).
set -u
mkdir -p gpurun_out/r06_b15
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_multirank.py \
  -m gpu -x -v --timeout 200 --timeout-method thread -k "panel" > gpurun_out/r06_b15/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06_b15/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06_b15/pytest.log | head; exit $rc; }
bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b15/hw 128 256 512 1024 2048 || exit 1
bash tools/r06_p8_comm.sh gpurun_out/r06_b15/p8 "shm 7" "shm 8" "rccl 8" || exit 1
