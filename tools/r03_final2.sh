# Session-2 final evidence: the default bench line (all sub-records, traffic from the committed
# PMC records), then the rocprofv3 kernel stats of the same command.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python bench.py > gpurun_out/r03f2_bench.json 2> gpurun_out/r03f2_bench.err; rc=$?
echo "bench rc=$rc"; tail -c 400 gpurun_out/r03f2_bench.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03f2_prof -o run -- \
  python3 bench.py > gpurun_out/r03f2_prof.log 2>&1; rc=$?
echo "prof rc=$rc"
rm -f gpurun_out/r03f2_prof/run_kernel_trace.csv
exit $rc
