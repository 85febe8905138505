#!/bin/bash
# round 5, batch 12: the per-rank size of the driver's N = 8 C4a point (n = 1.25e6) on one GPU —
# how far a block step's time sits above 1/8 of the n = 1e7 step (fixed per-step latency: small
# kernels, launch gaps), and which kernels carry it (rocprofv3 kernel trace).
set -u
mkdir -p gpurun_out/r05_b12
export TMPDIR=/tmp
for n in 1250000 2500000 5000000; do
  timeout -k 10 300 python bench.py --n $n --steps 5 --warmup 2 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0 \
    > gpurun_out/r05_b12/n$n.json 2> gpurun_out/r05_b12/n$n.err || exit 1
  python3 -c "
import json; l = json.loads(open('gpurun_out/r05_b12/n$n.json').read().strip().splitlines()[-1])
print($n, l['value'], l['ms_per_step'], {k: round(v, 2) for k, v in l['stage_ms_per_run'].items() if v})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_b12/kt -o kt --output-format csv -- python3 bench.py --n 1250000 --steps 2 --warmup 1 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0 > gpurun_out/r05_b12/kt.log 2>&1 || exit 1
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05_b12/kt/**/kt_kernel_stats.csv", recursive=True)[0]
rows = list(csv.DictReader(open(f)))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[:25]:
    print(f"{r['Name'][:70]:70s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.1f} us {float(r['TotalDurationNs'])/1e6:8.2f} ms")
print("total kernel ms", tot / 1e6)
PY
