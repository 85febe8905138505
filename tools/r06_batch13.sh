#!/bin/bash
# round 6, batch 13: (a) the P = 8 rehearsals with bench.py's shared-GPU queue cap
# (GPU_MAX_HW_QUEUES = 24 / 8 = 3); (b) the column-panel kernel's shape — rows per group and
# records per chunk load — forced per probe library (tools/variants/p<RPG>x<CH>) against the
# default choice, half-widths 128-2048.
set -u
export TMPDIR=/tmp
bash tools/r06_p8_comm.sh gpurun_out/r06_b13/p8 "shm 8" "rccl 8" || exit 1
bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b13/hw_default 128 256 512 1024 2048 || exit 1
for v in p8x32 p4x64 p8x16; do
  echo "== $v"
  RBL_LIB=$PWD/tools/variants/$v/librbl_hip.so bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b13/hw_$v 128 256 512 1024 2048 || exit 1
done
