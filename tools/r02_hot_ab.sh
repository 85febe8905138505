# R-MAT (C4b) SpMM with hot-first rows: tests, then bench lines for several hot-set sizes
# (RBL_HOT_COLS env override).  Usage: bash tools/r02_hot_ab.sh H1 [H2 ...]
set -u
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_rmat.py tests/test_gpu_memory_plan.py > gpurun_out/r02_t3.log 2>&1; rc=$?
echo "rmat tests rc=$rc"; tail -3 gpurun_out/r02_t3.log
[ $rc -ne 0 ] && exit $rc
for h in "$@"; do
  RBL_HOT_COLS=$h timeout -k 10 300 python bench.py --matrix rmat --steps 1 --warmup 1 --no-cpu-baseline \
    --no-ttk > gpurun_out/rmat_hot_$h.json 2> gpurun_out/rmat_hot_$h.err || exit $?
  python3 -c "import json;d=json.load(open('gpurun_out/rmat_hot_$h.json'));r=[x for x in (d['roofline'],d['roofline_secondary']) if 'spmm' in x['kernel']][0];print('hot $h', d['value'], 'iters/s', r['ms_per_launch'], 'ms/SpMM')"
done
