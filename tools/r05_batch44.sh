#!/bin/bash
# round 5, batch 44: pipelined Ritz with its side stream created and warmed by rbl_start — the
# Ritz / parity tests, the time-to-k probe serial vs pipelined, and the bench's time-to-k A/B.
set -u
mkdir -p gpurun_out/r05_b44
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_fullsize.py > gpurun_out/r05_b44/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b44/t.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error|assert" gpurun_out/r05_b44/t.log | head -30; exit $rc; }
for mode in 1 0; do
  for spec in planted slow; do
    echo "== RBL_RITZ_SERIAL=$mode $spec" >> gpurun_out/r05_b44/ttk.log
    if [ $mode = 1 ]; then export RBL_RITZ_SERIAL=1; else unset RBL_RITZ_SERIAL; fi
    RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ttk_probe.py $spec >> gpurun_out/r05_b44/ttk.log 2>&1 || { cat gpurun_out/r05_b44/ttk.log; exit 1; }
  done
done
grep -E "^==|total|^rep" gpurun_out/r05_b44/ttk.log
for rep in 1 2; do
  for mode in 1 0; do
    if [ $mode = 1 ]; then export RBL_RITZ_SERIAL=1; else unset RBL_RITZ_SERIAL; fi
    timeout -k 10 300 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --rmat-steps 0 --c3-steps 0 \
      > gpurun_out/r05_b44/ab_${mode}_$rep.json 2> gpurun_out/r05_b44/ab_${mode}_$rep.err || { tail -5 gpurun_out/r05_b44/ab_${mode}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b44/ab_${mode}_$rep.json').read().strip().splitlines()[-1])
t=d['time_to_k']; s=d['time_to_k_slow_spectrum']
print('serial=$mode', $rep, 'planted', t['seconds'], t['host_ms'], 'slow', s['seconds'], s['host_ms'])" | tee -a gpurun_out/r05_b44/ab.log
  done
done
