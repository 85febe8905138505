#!/bin/bash
# round 5, batch 47: the last tree's default line and the rocprofv3 kernel summary of the same command
set -u
mkdir -p gpurun_out/r05_b47
export TMPDIR=/tmp
timeout -k 10 600 python bench.py > gpurun_out/r05_b47/bench.json 2> gpurun_out/r05_b47/bench.err || { tail -5 gpurun_out/r05_b47/bench.err; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_b47/prof -o run --output-format csv -- python3 bench.py > gpurun_out/r05_b47/prof.json 2> gpurun_out/r05_b47/prof.err || { tail -5 gpurun_out/r05_b47/prof.err; exit 1; }
find gpurun_out/r05_b47/prof -name "*kernel_stats.csv"
python3 -c "
import json
for f in ('bench', 'prof'):
    d=json.loads(open('gpurun_out/r05_b47/%s.json' % f).read().strip().splitlines()[-1])
    print(f, d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['ms_per_run'], d['roofline_secondary']['ms_per_launch'], d['time_to_k']['seconds'], d['time_to_k_slow_spectrum']['seconds'])"
