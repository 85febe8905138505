# GPU round check: parity tests, then the bench, then a rocprofv3 kernel trace of the bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/t1.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/t1.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py --steps 2 > gpurun_out/b2.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 3000 gpurun_out/b2.log
if [ $rc -ne 0 ]; then exit $rc; fi
if [ "${PROFILE:-1}" = "1" ]; then
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ttk > gpurun_out/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"
fi
exit $rc
