#!/bin/bash
# round 5, batch 28: the pipelined Ritz vectors (row pieces, D2H behind them on a second stream):
# the new bit-identity test and the Ritz / speculation tests, then the time-to-k probe serial vs
# pipelined on both spectra.
set -u
mkdir -p gpurun_out/r05_b28
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_spill.py tests/test_gpu_fp32_basis.py > gpurun_out/r05_b28/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b28/t.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r05_b28/t.log | head -30; exit $rc; }
for mode in 1 0; do
  for spec in planted slow; do
    echo "== RBL_RITZ_SERIAL=$mode $spec" >> gpurun_out/r05_b28/ttk.log
    if [ $mode = 1 ]; then export RBL_RITZ_SERIAL=1; else unset RBL_RITZ_SERIAL; fi
    RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ttk_probe.py $spec >> gpurun_out/r05_b28/ttk.log 2>&1 || { cat gpurun_out/r05_b28/ttk.log; exit 1; }
  done
done
cat gpurun_out/r05_b28/ttk.log
