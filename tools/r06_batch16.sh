#!/bin/bash
# round 6, batch 16: where a column-panel step's time goes — wave 0 of workgroups 0 and 128
# stamps each phase of the step loop (s_memtime; tools/variants/stamps, and stamps15 = the same
# with FMAs, LDS reads, panel DMA and record loads removed) at H = 256 and 1024, one launch.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_b16
for v in stamps stamps15; do
  for H in 256 1024; do
    p=$(python3 -c "print(round(99 / (2 * $H), 6))")
    RBL_LIB=$PWD/tools/variants/$v/librbl_hip.so timeout -k 10 300 python bench.py --halfwidth $H --density $p \
      --steps 1 --warmup 0 --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk \
      > gpurun_out/r06_b16/${v}_hw$H.log 2> gpurun_out/r06_b16/${v}_hw$H.err; rc=$?
    echo "== $v H=$H rc=$rc"
    case $rc in 0|1) ;; *) exit $rc;; esac
    grep "panel stamps" gpurun_out/r06_b16/${v}_hw$H.log | sort | uniq -c | sort -rn | head -6
  done
done
