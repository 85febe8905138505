#!/bin/bash
# round 6, batch 26: fabric bytes of the shipped column-panel kernel (v9, residue-aligned panel
# order) at half-widths 1024 and 256 (FETCH_SIZE / WRITE_SIZE passes, tools/pmc_traffic_wl.sh),
# against v4's 22.6 / 20 GB per launch (profiles/r06_panel_v4_pmc_b12.txt).
set -u
for H in 1024 256; do
  p=$(python3 -c "print(round(99 / (2 * $H), 6))")
  bash tools/pmc_traffic_wl.sh wide$H --halfwidth $H --density $p --wide-steps 0 || exit 1
  python3 tools/pmc_summarize.py gpurun_out/pmc_wide$H - "hashwindow 10000000 32 38" | grep -iE "panel|calib" || true
done
