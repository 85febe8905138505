# Round-3 final evidence: PMC HBM traffic of the current kernels (C4a, separate FETCH_SIZE /
# WRITE_SIZE passes + calibration), then the default bench line priced with it, then the
# rocprofv3 kernel stats of the same bench command.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py \
  tests/test_gpu_golden.py tests/test_gpu_parity.py > gpurun_out/r03f_tests.log 2>&1 || { echo "tests failed"; tail -5 gpurun_out/r03f_tests.log; exit 1; }
tail -1 gpurun_out/r03f_tests.log
bash tools/pmc_traffic.sh > gpurun_out/r03f_pmc.log 2>&1 || { echo "pmc failed"; tail -5 gpurun_out/r03f_pmc.log; exit 1; }
python tools/pmc_summarize.py gpurun_out/pmc gpurun_out/pmc_traffic_r03.json > gpurun_out/r03f_pmc_summary.txt || exit 1
cat gpurun_out/r03f_pmc_summary.txt
rm -rf gpurun_out/pmc/*/*.db
timeout -k 10 900 python bench.py --traffic-json gpurun_out/pmc_traffic_r03.json > gpurun_out/r03f_bench.json 2> gpurun_out/r03f_bench.err; rc=$?
echo "bench rc=$rc"; tail -c 600 gpurun_out/r03f_bench.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03f_prof -o run -- \
  python3 bench.py --traffic-json gpurun_out/pmc_traffic_r03.json > gpurun_out/r03f_prof.log 2>&1; rc=$?
echo "prof rc=$rc"
rm -f gpurun_out/r03f_prof/run_kernel_trace.csv
exit $rc
