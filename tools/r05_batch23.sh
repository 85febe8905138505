#!/bin/bash
# round 5, batch 23: the parity file (incl. the latency-knob test) after the per-call chunk knob
set -u
mkdir -p gpurun_out/r05_b23
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_multirank.py > gpurun_out/r05_b23/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b23/t.log)"
grep -E "FAILED|Error|latency_knobs" gpurun_out/r05_b23/t.log | head -20
exit $rc
