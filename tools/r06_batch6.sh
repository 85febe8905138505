#!/bin/bash
# round 6, batch 6: column-panel SpMM with non-temporal CSR loads — time per launch at
# half-widths 128-2048 and the fabric bytes / L2 hit rate at 1024.
set -u
export TMPDIR=/tmp
bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b6/hw 128 256 512 1024 2048 || exit 1
H=1024; p=$(python3 -c "print(round(99 / (2 * $H), 6))")
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r06_b6/pmc_hw$H/g4 -o p -- \
  python3 bench.py --halfwidth $H --density $p --steps 1 --warmup 0 --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk \
  > gpurun_out/r06_b6/pmc1.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/r06_b6/pmc_hw$H/g5 -o p -- \
  python3 bench.py --halfwidth $H --density $p --steps 1 --warmup 0 --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk \
  > gpurun_out/r06_b6/pmc2.log 2>&1 || exit 1
python3 tools/pmc_groups_summary.py gpurun_out/r06_b6/pmc_hw$H k_spmm_panel | grep -E "==|memory"
