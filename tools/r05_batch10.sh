#!/bin/bash
# round 5, batch 10: the CPU baseline's fixed-step form at the headline's own n (n = 1e7: the
# oracle's rbl_start + first 8 block steps), beside the default sample, in one bench run.
set -u
mkdir -p gpurun_out
timeout -k 10 1100 python bench.py --steps 1 --warmup 1 --rmat-steps 0 --c3-steps 0 --no-ttk-slow \
  --cpu-fixed-n 10000000 > gpurun_out/r05_bench_cpu_fixed_n1e7.json 2> gpurun_out/r05_bench_cpu_fixed_n1e7.err
rc=$?; echo "rc=$rc"; grep "^\[bench" gpurun_out/r05_bench_cpu_fixed_n1e7.err | tail -3
tail -c 1500 gpurun_out/r05_bench_cpu_fixed_n1e7.json
exit $rc
