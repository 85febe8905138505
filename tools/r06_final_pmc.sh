#!/bin/bash
# round 6: PMC evidence for the default line's kernels — FETCH_SIZE / WRITE_SIZE passes with
# the per-width calibration probe (tools/pmc_traffic.sh), then the held-clock pass (GRBM).
set -u
export TMPDIR=/tmp
bash tools/pmc_traffic.sh || exit $?
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc_clk -o c -- \
  python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0 > gpurun_out/pmc_clk.log 2>&1 || exit $?
python3 tools/pmc_summarize.py gpurun_out/pmc gpurun_out/pmc/summary.json | tail -3
echo done
