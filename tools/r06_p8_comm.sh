#!/bin/bash
# round 6: the P = 8 collective collapse of the one-GPU rehearsal.
# The default C4a job at n = 1e7, C4a runs only, on P processes sharing the one GPU over the
# shm transport or over RCCL (one host id per rank: the socket transport on loopback); each
# line carries every rank's collectives (host / device time per call), stage split, the CPU
# time its process used, the cgroup's CPU quota and throttling, and the GPU processes KFD knows.
# Usage: tools/r06_p8_comm.sh <outdir> "shm 8" "rccl 8" ...
set -u
out=${1:-gpurun_out/r06_p8}; shift
mkdir -p $out
export TMPDIR=/tmp
echo "cpus in affinity: $(python3 -c 'import os; print(len(os.sched_getaffinity(0)))') of $(nproc --all)"
echo "cgroup cpu.max: $(cat /sys/fs/cgroup/cpu.max 2>/dev/null || echo n/a)"
for p in hws_max_conc_proc sched_policy mes cwsr_enable; do
  echo "amdgpu.$p = $(cat /sys/module/amdgpu/parameters/$p 2>/dev/null || echo n/a)"
done
echo "KFD processes before the runs: $(ls /sys/class/kfd/kfd/proc 2>/dev/null | wc -l)"
common="--steps 2 --warmup 1 --rmat-steps 0 --c3-steps 0 --c5-steps 0 --no-cpu-baseline --no-ttk"
for cfg in "$@"; do
  set -- $cfg
  tr=$1; P=$2; shift 2
  [ $tr = rccl ] && export RBL_RCCL_HOST_PER_RANK=1 || unset RBL_RCCL_HOST_PER_RANK
  NCCL_DEBUG=WARN timeout -k 20 400 python bench.py --gpus $P --transport $tr $common "$@" \
    > $out/${tr}${P}.json 2> $out/${tr}${P}.err; rc=$?
  echo "$tr P=$P rc=$rc"
  [ $rc -ne 0 ] && { tail -30 $out/${tr}${P}.err; exit $rc; }
  python3 tools/r06_p8_summary.py $out/${tr}${P}.json
done
