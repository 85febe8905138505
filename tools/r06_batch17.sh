#!/bin/bash
# round 6, batch 17: column-panel v6 (epilogue four rows per B_i^T read, conditional LDS
# read-ahead in groups of 2 / 4) — tests, the half-width sweep, and the phase stamps.
set -u
mkdir -p gpurun_out/r06_b17
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_multirank.py \
  -m gpu -x -v --timeout 200 --timeout-method thread -k "panel" > gpurun_out/r06_b17/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06_b17/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06_b17/pytest.log | head; exit $rc; }
bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b17/hw 128 256 512 1024 2048 || exit 1
for H in 256 1024; do
  p=$(python3 -c "print(round(99 / (2 * $H), 6))")
  RBL_LIB=$PWD/tools/variants/stamps/librbl_hip.so timeout -k 10 300 python bench.py --halfwidth $H --density $p \
    --steps 1 --warmup 0 --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk \
    > gpurun_out/r06_b17/stamps_hw$H.log 2> gpurun_out/r06_b17/stamps_hw$H.err || exit 1
done
