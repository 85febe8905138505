#!/bin/bash
# round 5, batch 22: evidence on the final tree — the whole -m gpu suite, the default bench line,
# and the headline (C4a only) under rocprofv3 --kernel-trace --stats, whose kernel averages the
# line's roofline must agree with.
set -u
mkdir -p gpurun_out/r05_b22
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread tests \
  > gpurun_out/r05_b22/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b22/t.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r05_b22/t.log | head -20; exit $rc; }
timeout -k 10 600 python bench.py > gpurun_out/r05_b22/bench.json 2> gpurun_out/r05_b22/bench.err || { tail -5 gpurun_out/r05_b22/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b22/bench.json').read().strip().splitlines()[-1])
print('default', d['value'], d['ms_per_step'], d['stage_pass_ms_per_run'], d['roofline']['frac'], d['roofline']['ms_per_run'], d['roofline_secondary']['frac'], d['roofline_secondary']['ms_per_launch'])
print('c4b', d['c4b_rmat']['value'], 'c3', d['c3_circuit']['value'], 'cpu', d['cpu_baseline']['value'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_b22/kt -o kt --output-format csv -- python3 bench.py --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0 > gpurun_out/r05_b22/kt.json 2> gpurun_out/r05_b22/kt.err || exit 1
python3 - <<'PY'
import csv, glob, json
f = glob.glob("gpurun_out/r05_b22/kt/**/kt_kernel_stats.csv", recursive=True)[0]
d = json.loads(open("gpurun_out/r05_b22/kt.json").read().strip().splitlines()[-1])
print("line:", d["value"], "reorth ms/run", d["roofline"]["ms_per_run"], "spmm ms/launch", d["roofline_secondary"]["ms_per_launch"])
for r in sorted(csv.DictReader(open(f)), key=lambda r: -float(r["TotalDurationNs"]))[:12]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):6d} {float(r['AverageNs'])/1e3:10.1f} us {float(r['TotalDurationNs'])/1e6:10.2f} ms")
PY
