#!/bin/bash
# round 5, second GPU batch: the b = 16 partial-reorth kernels on the C3 shape (reorth_probe at
# n = 1,585,478, b = 16, basis 2..72 panels: C3's even steps) — kernel-trace stats and the
# occupancy / MFMA / stall / traffic counter groups (one rocprofv3 --pmc pass each); then the
# driver's N = 8 point rehearsed over RCCL on this one GPU (every rank its own RCCL host).
set -u
mkdir -p gpurun_out/r05_b16
export TMPDIR=/tmp
P=tools/reorth_probe
A="1585478 16 72"
timeout -k 10 120 $P $A > gpurun_out/r05_b16/probe.log 2>&1; rc=$?
echo "probe rc=$rc"; tail -2 gpurun_out/r05_b16/probe.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_b16/kt -o kt --output-format csv -- $P $A > gpurun_out/r05_b16/kt.log 2>&1; rc=$?
echo "kernel trace rc=$rc"
[ $rc -ne 0 ] && exit $rc
PMC_TCC=1 bash tools/pmc_groups.sh gpurun_out/r05_b16/pmc $P $A; rc=$?
echo "pmc rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 tools/pmc_groups_summary.py gpurun_out/r05_b16/pmc k_ > gpurun_out/r05_b16/pmc_summary.txt 2>&1
cat gpurun_out/r05_b16/pmc_summary.txt | head -40
if [ "${RCCL8:-1}" = 1 ]; then
  RBL_RCCL_HOST_PER_RANK=1 NCCL_DEBUG=WARN timeout -k 20 900 python bench.py --gpus 8 --n 2000000 \
    --steps 2 --warmup 1 --rmat-steps 2 --c3-steps 2 --c5-n 8000000 --c5-steps 1 \
    > gpurun_out/r05_bench_rccl8.json 2> gpurun_out/r05_bench_rccl8.err; rc=$?
  echo "rccl8 bench rc=$rc"; tail -c 600 gpurun_out/r05_bench_rccl8.json
fi
exit $rc
