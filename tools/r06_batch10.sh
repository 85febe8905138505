#!/bin/bash
# round 6, batch 10: the whole -m gpu suite on the current tree, then the P = 8 rehearsals with
# bench.py's shared-GPU queue cap (GPU_MAX_HW_QUEUES = 24 / ranks per GPU = 3 at P = 8).
set -u
export TMPDIR=/tmp
bash tools/r06_gpu_tests.sh gpurun_out/r06_b10/tests || exit 1
bash tools/r06_p8_comm.sh gpurun_out/r06_b10/p8 "shm 8" "rccl 8" || exit 1
