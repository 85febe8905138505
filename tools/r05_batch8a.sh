#!/bin/bash
# round 5: the whole -m gpu suite (C4a and C4b against their full-size oracle fixtures included),
# then the same suite with the two-waves-per-SIMD band SpMM (RBL_BT2=1).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r05_test_gpu_full.log 2>&1; rc=$?
echo "full rc=$rc: $(tail -1 gpurun_out/r05_test_gpu_full.log)"
[ $rc -ne 0 ] && exit $rc
RBL_BT2=1 timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 400 --timeout-method thread > gpurun_out/r05_test_gpu_bt2_on.log 2>&1; rc=$?
echo "bt2 rc=$rc: $(tail -1 gpurun_out/r05_test_gpu_bt2_on.log)"
exit $rc
