#!/bin/bash
# round 5, batch 11: BASELINE config 5 at the per-rank sizes of the driver's N = 2 and N = 4
# points (n = 2.5e7 / 1.25e7 rows, fp32 basis, CSR released) on one GPU, after the C3 sub-record
# as in the driver's job (so the HBM preflight sees what the job leaves allocated).
set -u
mkdir -p gpurun_out
for n in 25000000 12500000; do
  timeout -k 10 600 python bench.py --n 1000000 --steps 1 --warmup 1 --rmat-steps 0 --c3-steps 1 \
    --no-cpu-baseline --no-ttk-slow --c5-min-ranks 1 --c5-n $n --c5-steps 2 \
    > gpurun_out/r05_bench_c5_n$n.json 2> gpurun_out/r05_bench_c5_n$n.err
  rc=$?; echo "c5 n=$n rc=$rc"
  [ $rc -ne 0 ] && { tail -5 gpurun_out/r05_bench_c5_n$n.err; exit $rc; }
  python3 -c "
import json; l = json.loads(open('gpurun_out/r05_bench_c5_n$n.json').read().strip().splitlines()[-1]); c = l['c5_mixed']
print({k: c.get(k) for k in ('value', 'ms_per_step', 'skipped', 'error', 'time_to_k')})"
done
