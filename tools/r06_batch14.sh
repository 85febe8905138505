#!/bin/bash
# round 6, batch 14: (a) the P = 8 rehearsals with the shared-GPU queue cap (bench.py lowers the
# box's GPU_MAX_HW_QUEUES=4 to 24 / 8 = 3); (b) what each part of the column-panel kernel costs:
# probe libraries with parts removed (tools/variants/abl<mask>: 1 FMAs, 2 LDS reads, 4 panel DMA,
# 8 record loads; wrong results, timing only) at H = 256 and 1024, against the product library.
set -u
export TMPDIR=/tmp
bash tools/r06_p8_comm.sh gpurun_out/r06_b14/p8 "shm 8" "rccl 8" || exit 1
for v in default abl1 abl2 abl3 abl4 abl8 abl12 abl15; do
  lib=""
  [ $v != default ] && lib=$PWD/tools/variants/$v/librbl_hip.so
  echo "== $v"
  RBL_LIB=$lib bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b14/hw_$v 256 1024; rc=$?
  case $rc in 0|1) ;; *) echo "stop: rc=$rc"; exit $rc;; esac
done
