# Round-3 check 2: circuit generator + C3/C4b fixtures + full-size C4b + tier / split tests,
# one default bench line, then the column-tier A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 400 --timeout-method thread \
  tests/test_gpu_circuit.py tests/test_gpu_rmat.py tests/test_gpu_c2_c3.py \
  tests/test_gpu_rmat_fullsize.py tests/test_gpu_multirank.py tests/test_gpu_parity.py tests/test_lib_host.py \
  > gpurun_out/r03_t2.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -8 gpurun_out/r03_t2.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py > gpurun_out/r03_bench2.json 2> gpurun_out/r03_bench2.err; rc=$?
echo "bench rc=$rc"; tail -c 1500 gpurun_out/r03_bench2.json
[ $rc -ne 0 ] && exit $rc
bash tools/r03_tiers_ab.sh
