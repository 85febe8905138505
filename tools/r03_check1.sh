# Round-3 first check: the SpMM option remap, the C4b tests (oracle fixture at n = 1e6, full-size
# properties at n = 1e7), then one default bench line (C4a + the c4b_rmat sub-record).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread \
  tests/test_gpu_spmm.py tests/test_gpu_rmat.py tests/test_gpu_circuit.py tests/test_gpu_c2_c3.py \
  tests/test_gpu_rmat_fullsize.py \
  > gpurun_out/r03_t1.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -8 gpurun_out/r03_t1.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r03_bench1.json 2> gpurun_out/r03_bench1.err; rc=$?
echo "bench rc=$rc"; tail -c 3000 gpurun_out/r03_bench1.json
exit $rc
