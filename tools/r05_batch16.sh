#!/bin/bash
# round 5, batch 16: the shifted-third-pass local-reorth Gram test (k_cloc_rinv), with prints
set -u
mkdir -p gpurun_out/r05_b16
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v -s --timeout 200 --timeout-method thread tests/test_gpu_parity.py \
  -k "shifted_third_pass or pass_fusions or cholqr" > gpurun_out/r05_b16/t.log 2>&1; rc=$?
grep -E "statuses|PASSED|FAILED|assert|Error" gpurun_out/r05_b16/t.log | head -40
exit $rc
