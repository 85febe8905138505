#!/bin/bash
# round 5, batch 24: the Ritz path — pinned staging slots allocated by rbl_start, LDS-tiled
# transposes — the whole -m gpu suite, the time-to-k probe with the Ritz trace, the default line.
set -u
mkdir -p gpurun_out/r05_b24
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread tests \
  > gpurun_out/r05_b24/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b24/t.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r05_b24/t.log | head -20; exit $rc; }
RBL_RITZ_TRACE=1 timeout -k 10 200 python -u tools/r05_ttk_probe.py > gpurun_out/r05_b24/ttk.log 2>&1 || exit 1
cat gpurun_out/r05_b24/ttk.log
timeout -k 10 600 python bench.py > gpurun_out/r05_b24/bench.json 2> gpurun_out/r05_b24/bench.err || { tail -5 gpurun_out/r05_b24/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b24/bench.json').read().strip().splitlines()[-1])
print('default', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline_secondary']['frac'])
print('ttk', d['time_to_k']['seconds'], d['time_to_k']['host_ms'], 'slow', d['time_to_k_slow_spectrum']['seconds'], d['time_to_k_slow_spectrum']['host_ms'])
print('c4b', d['c4b_rmat']['value'], 'c3', d['c3_circuit']['value'])"
