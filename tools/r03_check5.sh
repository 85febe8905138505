# Full -m gpu suite on the current tree, then smoke().
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -x --timeout 600 --timeout-method thread \
  > gpurun_out/r03_check5_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/r03_check5_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
# b = 16 partial-reorth rates at C3's n (diagnostic)
timeout -k 10 180 ./tools/reorth_probe 1585478 16 72 > gpurun_out/r03_probe_b16.log 2>&1 && tail -1 gpurun_out/r03_probe_b16.log
timeout -k 10 180 ./tools/reorth_probe 1000000 16 74 > gpurun_out/r03_probe_b16_c2.log 2>&1 && tail -1 gpurun_out/r03_probe_b16_c2.log
