#!/bin/bash
# round 5 evidence: the default bench line, the rocprofv3 kernel-trace summary of the same
# command, PMC traffic (FETCH_SIZE / WRITE_SIZE passes) and clock passes (tools/round_profile.sh),
# then C5 at the per-rank size of the driver's N = 2 point on one GPU (n = 2.5e7).
set -u
bash tools/round_profile.sh r05 || exit $?
python3 tools/pmc_summarize.py gpurun_out/pmc gpurun_out/pmc_traffic_r05.json > gpurun_out/pmc_summary_r05.txt 2>&1 || exit 1
timeout -k 10 600 python bench.py --steps 1 --warmup 1 --rmat-steps 0 --c3-steps 0 --no-cpu-baseline \
  --no-ttk-slow --c5-min-ranks 1 --c5-n 25000000 --c5-steps 2 > gpurun_out/r05_bench_c5_n25e6.json 2> gpurun_out/r05_bench_c5_n25e6.err
rc=$?; echo "c5 per-rank N=2 rc=$rc"; tail -c 400 gpurun_out/r05_bench_c5_n25e6.json
exit $rc
