#!/bin/bash
# round 6, batch 29: column panels <4, 48> (48-record chunks: a row's ~50 entries per panel at
# H = 128-256 in one chunk instead of a 32-record chunk + a reload; the early Q_{i-1} loads
# dropped for chunks > 32 to stay at 128 VGPRs) — tools/variants/p448 forces it — against the
# product's automatic <4, 32> at H = 128, 256, 512; panel tests on the variant first.
set -u
mkdir -p gpurun_out/r06_b29
export TMPDIR=/tmp
RBL_LIB=tools/variants/p448/librbl_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_multirank.py \
  -m gpu -x -q --timeout 200 --timeout-method thread -k "panel" > gpurun_out/r06_b29/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06_b29/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06_b29/pytest.log | head; exit $rc; }
for rep in 1 2; do
  echo "== product <4,32>, rep $rep"
  bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b29/p$rep 128 256 512 || exit 1
  echo "== <4,48>, rep $rep"
  RBL_LIB=tools/variants/p448/librbl_hip.so bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b29/v$rep 128 256 512 || exit 1
done
