# Round-2 feature check: new GPU tests (memory plan, fp32 spill / any b, Ritz chunks), the C5
# full-size test at n = 5e7, then a C5 bench line.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_spill.py \
  > gpurun_out/r02_t1.log 2>&1; rc=$?
echo "new tests rc=$rc"; tail -5 gpurun_out/r02_t1.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 800 --timeout-method thread \
  tests/test_gpu_c5.py > gpurun_out/r02_c5.log 2>&1; rc=$?
echo "c5 test rc=$rc"; tail -5 gpurun_out/r02_c5.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python bench.py --n 50000000 --basis-bits 32 --keep-csr 0 --device-blocks -1 \
  --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/r02_bench_c5.json 2> gpurun_out/r02_bench_c5.err; rc=$?
echo "bench c5 rc=$rc"; tail -c 2500 gpurun_out/r02_bench_c5.json
exit $rc
