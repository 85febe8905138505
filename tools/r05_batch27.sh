#!/bin/bash
# round 5, batch 27: graded residual-driven speculation as the default (1 step in the uncertain
# zone) — the whole -m gpu suite (multi-rank and multi-process runs now speculate too), the
# slow-spectrum time-to-k probe, the default line.
set -u
mkdir -p gpurun_out/r05_b27
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread tests \
  > gpurun_out/r05_b27/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b27/t.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r05_b27/t.log | head -20; exit $rc; }
timeout -k 10 200 python -u tools/r05_ttk_probe.py slow > gpurun_out/r05_b27/ttk.log 2>&1 || { cat gpurun_out/r05_b27/ttk.log; exit 1; }
cat gpurun_out/r05_b27/ttk.log
timeout -k 10 600 python bench.py > gpurun_out/r05_b27/bench.json 2> gpurun_out/r05_b27/bench.err || { tail -5 gpurun_out/r05_b27/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b27/bench.json').read().strip().splitlines()[-1])
print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_secondary']['frac'])
t=d['time_to_k']; s=d['time_to_k_slow_spectrum']
print('ttk', t['seconds'], t['host_ms'], t['speculated_steps'], 'slow', s['seconds'], s['host_ms'], s['speculated_steps'], s['speculated_discarded'])
print('c4b', d['c4b_rmat']['value'], 'c3', d['c3_circuit']['value'])"
