#!/bin/bash
# round 5, batch 26: residual-driven speculation (rbl.lanczos speculate="auto", the new default):
# the parity of speculative runs, then the C4a time-to-k probe strict vs auto on both spectra.
set -u
mkdir -p gpurun_out/r05_b26
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py > gpurun_out/r05_b26/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b26/t.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r05_b26/t.log | head -20; exit $rc; }
for mode in 0 auto; do
  for spec in planted slow; do
    echo "== TTK_SPEC=$mode $spec" >> gpurun_out/r05_b26/ttk.log
    TTK_SPEC=$mode timeout -k 10 200 python -u tools/r05_ttk_probe.py $spec >> gpurun_out/r05_b26/ttk.log 2>&1 || { cat gpurun_out/r05_b26/ttk.log; exit 1; }
  done
done
cat gpurun_out/r05_b26/ttk.log
