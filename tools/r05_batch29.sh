#!/bin/bash
# round 5, batch 29: why the pipelined Ritz is slower on the slow spectrum (28 blocks): kernel +
# memory-copy traces of the time-to-k probe, serial vs pipelined.
set -u
mkdir -p gpurun_out/r05_b29
export TMPDIR=/tmp
for mode in 1 0; do
  if [ $mode = 1 ]; then export RBL_RITZ_SERIAL=1; else unset RBL_RITZ_SERIAL; fi
  RBL_RITZ_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv \
    -d gpurun_out/r05_b29/prof_s$mode -o run -- python3 tools/r05_ttk_probe.py slow > gpurun_out/r05_b29/probe_s$mode.log 2>&1 || { tail -20 gpurun_out/r05_b29/probe_s$mode.log; exit 1; }
done
cat gpurun_out/r05_b29/probe_s*.log | grep -v "^W2026\|rocprofiler" | tail -20
find gpurun_out/r05_b29 -name "*.csv" | head
