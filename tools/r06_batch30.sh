#!/bin/bash
# round 6, batch 30: the column-panel shapes forced one at a time (<8,16>, <4,32>, <4,48>;
# tools/variants/p816, p432, p448) at H = 128 .. 2048, two alternations — to set the shape rule.
set -u
mkdir -p gpurun_out/r06_b30
export TMPDIR=/tmp
for rep in 1 2; do
  for v in p816 p432 p448; do
    echo "== $v, rep $rep"
    RBL_LIB=tools/variants/$v/librbl_hip.so bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b30/$v$rep 128 256 512 768 1024 2048 || exit 1
  done
done
