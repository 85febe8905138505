bash tools/r06_p8_comm.sh gpurun_out/r06_p8b "shm 6" "shm 7" "shm 8" "rccl 7" "rccl 8" && bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_hw0
