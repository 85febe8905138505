#!/bin/bash
# round 5, batch 25: the Ritz chunks in the run scratch (no per-call allocation), and the
# slow-spectrum bench fix — the whole -m gpu suite, the time-to-k probe with the Ritz trace, the default line.
set -u
mkdir -p gpurun_out/r05_b25
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread tests \
  > gpurun_out/r05_b25/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b25/t.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r05_b25/t.log | head -20; exit $rc; }
RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ttk_probe.py > gpurun_out/r05_b25/ttk.log 2>&1 && RBL_RITZ_TRACE=1 timeout -k 10 250 python -u tools/r05_ttk_probe.py slow >> gpurun_out/r05_b25/ttk.log 2>&1 || exit 1
cat gpurun_out/r05_b25/ttk.log
RBL_RITZ_TRACE=1 timeout -k 10 600 python bench.py > gpurun_out/r05_b25/bench.json 2> gpurun_out/r05_b25/bench.err || { tail -5 gpurun_out/r05_b25/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b25/bench.json').read().strip().splitlines()[-1])
print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_secondary']['frac'])
print('ttk', d['time_to_k']['seconds'], d['time_to_k']['host_ms'], 'slow', d['time_to_k_slow_spectrum']['seconds'], d['time_to_k_slow_spectrum']['host_ms'])
print('c4b', d['c4b_rmat']['value'], 'c3', d['c3_circuit']['value'])"
grep rbl_ritz gpurun_out/r05_b25/bench.err
