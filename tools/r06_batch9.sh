#!/bin/bash
# round 6, batch 9: (a) the P = 8 controls of VERDICT r05 item 1 — shm at P = 6, 7, 8, and
# shm / RCCL at P = 8 with one hardware queue per process (GPU_MAX_HW_QUEUES=1: if the collapse
# is the eight processes' queues oversubscribing the one GPU's scheduler, this restores it);
# (b) column-panel SpMM with the CSR stream loaded nt (librbl_hip_nt.so) against the default
# policy, A/B/A at H = 256 and 1024.
set -u
export TMPDIR=/tmp
bash tools/r06_p8_comm.sh gpurun_out/r06_b9/p8 "shm 6" "shm 7" "shm 8" || exit 1
GPU_MAX_HW_QUEUES=1 bash tools/r06_p8_comm.sh gpurun_out/r06_b9/p8q1 "shm 8" "rccl 8" || exit 1
lib=gpu-randomized-block-lanczos_amd/rbl
bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b9/hwA 256 1024 || exit 1
RBL_LIB=$PWD/$lib/librbl_hip_nt.so bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b9/hwNT 256 1024 || exit 1
bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b9/hwA2 256 1024 || exit 1
