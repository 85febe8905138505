#!/bin/bash
# round 6, batch 19: the LDS-window kernel (2) against the column panels (7) where both apply
# (half-widths 72-120: a 16-row tile's window within the 256-row ring), forced, n = 1e7 ~100/row.
set -u
export TMPDIR=/tmp
for H in 72 96 120; do
  for k in 2 7; do
    echo "== kernel $k"
    bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b19/hw_k$k $H -- --spmm-kernel $k || exit 1
  done
done
