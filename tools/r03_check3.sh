# Round-3 check 3: the indexed halo (multi-rank unbanded) and everything multi-rank, then a
# quick R-MAT line at one rank (unchanged path) and the comm counts at 8 in-process ranks.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_rmat.py tests/test_gpu_multirank.py tests/test_gpu_circuit.py tests/test_gpu_c2_c3.py \
  > gpurun_out/r03_t3.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -5 gpurun_out/r03_t3.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/r03_comm_counts.py 8 > gpurun_out/r03_comm_counts.log 2>&1; rc=$?
echo "comm counts rc=$rc"; tail -3 gpurun_out/r03_comm_counts.log | cut -c1-300
exit $rc
