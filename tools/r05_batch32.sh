#!/bin/bash
# round 5, batch 32: does the bench's full stage timing (RBL_OPT_TIMERS 1) inflate its slow-spectrum
# time-to-k (Ritz + D2H ~70 ms in the bench vs ~50 in the probe)?  The probe with and without timers.
set -u
mkdir -p gpurun_out/r05_b32
export TMPDIR=/tmp
for t in "" timers "" timers; do
  echo "== slow $t" >> gpurun_out/r05_b32/ttk.log
  RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ttk_probe.py slow $t >> gpurun_out/r05_b32/ttk.log 2>&1 || { cat gpurun_out/r05_b32/ttk.log; exit 1; }
done
cat gpurun_out/r05_b32/ttk.log
