#!/bin/bash
# round 5, batch 43: the pipelined Ritz again, kernels on a side stream and the copies on the
# context's stream — the bit-identity test, then the time-to-k probe serial vs pipelined (both
# spectra), then the bench-order probe.
set -u
mkdir -p gpurun_out/r05_b43
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py -k "ritz or speculative or golden" > gpurun_out/r05_b43/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b43/t.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r05_b43/t.log | head -30; exit $rc; }
for mode in 1 0 1 0; do
  for spec in planted slow; do
    echo "== RBL_RITZ_SERIAL=$mode $spec" >> gpurun_out/r05_b43/ttk.log
    if [ $mode = 1 ]; then export RBL_RITZ_SERIAL=1; else unset RBL_RITZ_SERIAL; fi
    RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ttk_probe.py $spec >> gpurun_out/r05_b43/ttk.log 2>&1 || { cat gpurun_out/r05_b43/ttk.log; exit 1; }
  done
done
grep -E "^==|total" gpurun_out/r05_b43/ttk.log
