# Full -m gpu suite after the seg-kernel change (B_i in LDS at b = 32), smoke, the default bench
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread \
  > gpurun_out/r03_check6_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r03_check6_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" || exit 1
timeout -k 10 900 python bench.py > gpurun_out/r03c6_bench.json 2> gpurun_out/r03c6_bench.err; rc=$?
echo "bench rc=$rc"
exit $rc
