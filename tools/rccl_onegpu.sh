#!/bin/bash
# Two RCCL ranks on GPU 0 (tests/rccl_rank.py: one host id per rank, loopback sockets), a
# hash-window and an R-MAT push/pull case; logs and npz under gpurun_out/.
set -u
mkdir -p gpurun_out
uid=/tmp/rbl_rccl_uid_$$
rm -f $uid
CASES='[{"name":"hw","matrix":"hashwindow","n":9000,"W":64,"p":0.7734,"seed":41,"b":32,"steps":10},{"name":"rmat_push","matrix":"rmat","n":60000,"scale":16,"edges":3960000,"seed":7,"b":32,"steps":10,"push":1}]'
export NCCL_DEBUG=${NCCL_DEBUG:-WARN}
timeout -k 5 150 python -u tests/rccl_rank.py --uid-file $uid --nranks 2 --rank 0 --cases "$CASES" \
  --out gpurun_out/rccl0.npz > gpurun_out/rccl0.log 2>&1 &
p0=$!
timeout -k 5 150 python -u tests/rccl_rank.py --uid-file $uid --nranks 2 --rank 1 --cases "$CASES" \
  --out gpurun_out/rccl1.npz > gpurun_out/rccl1.log 2>&1
rc1=$?
wait $p0
rc0=$?
rm -f $uid
echo "rank0 rc=$rc0 rank1 rc=$rc1"
tail -5 gpurun_out/rccl0.log gpurun_out/rccl1.log
[ $rc0 -eq 0 ] && [ $rc1 -eq 0 ]
