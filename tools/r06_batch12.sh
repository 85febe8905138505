#!/bin/bash
# round 6, batch 12 (panel v4: panel-major records): counters of the column-panel SpMM at half-widths 256 and 1024 (C4a-sized):
# instruction mix, waits, LDS, L2 hits and fabric bytes (one --pmc pass per group).
set -u
export TMPDIR=/tmp
for H in 1024 256; do
  p=$(python3 -c "print(round(99 / (2 * $H), 6))")
  PMC_TCC=1 bash tools/pmc_groups.sh gpurun_out/r06_b12/pmc_hw$H python3 bench.py --halfwidth $H --density $p \
    --steps 1 --warmup 0 --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk || exit 1
  python3 tools/pmc_groups_summary.py gpurun_out/r06_b12/pmc_hw$H k_spmm_panel
done
