#!/bin/bash
# round 5, batch 54: the final tree (row-piece Ritz on the fp32 basis too) — the whole -m gpu suite, smoke(), the default line.
set -u
mkdir -p gpurun_out/r05_b54
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread tests \
  > gpurun_out/r05_b54/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b54/t.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r05_b54/t.log | head -20; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r05_b54/smoke.log 2>&1 || { cat gpurun_out/r05_b54/smoke.log; exit 1; }
tail -2 gpurun_out/r05_b54/smoke.log
timeout -k 10 600 python bench.py > gpurun_out/r05_b54/bench.json 2> gpurun_out/r05_b54/bench.err || { tail -5 gpurun_out/r05_b54/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b54/bench.json').read().strip().splitlines()[-1])
print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_secondary']['frac'])
t=d['time_to_k']; s=d['time_to_k_slow_spectrum']
print('ttk', t['seconds'], 'slow', s['seconds'], s['speculated_steps'], s['speculated_discarded'])
print('c4b', d['c4b_rmat']['value'], 'c3', d['c3_circuit']['value'], 'cpu', d['cpu_baseline']['value'])"
