# Round-3 check 4: the full GPU suite on the current tree, then the mixed-mode lines (C4a with the
# fp32 basis, and C5 at n = 5e7 on one GPU with host spill) after the 32x32x2 fp32 kernels.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/r03c4_tests.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/r03c4_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python bench.py --basis-bits 32 --steps 5 --warmup 1 --rmat-steps 0 --c3-steps 0 --no-cpu-baseline \
  > gpurun_out/r03c4_mixed.json 2> gpurun_out/r03c4_mixed.err || exit 1
tail -c 300 gpurun_out/r03c4_mixed.json; echo
timeout -k 10 600 python bench.py --n 50000000 --basis-bits 32 --keep-csr 0 --device-blocks -1 \
  --steps 1 --warmup 1 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0 > gpurun_out/r03c4_c5.json 2> gpurun_out/r03c4_c5.err || exit 1
tail -c 300 gpurun_out/r03c4_c5.json
