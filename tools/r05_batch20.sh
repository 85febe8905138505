#!/bin/bash
# round 5, batch 20 (rerun with the mask-free sweep: the parity, multirank, fp32-basis and
# restarted files instead of the whole suite): the Cholesky on both halves of the wave (k_chol_elim2) and the wide slab
# reduction (k_reduce_wide): the whole -m gpu suite, then an A/B at the per-rank N = 8 size
# against the previous kernels (RBL_CHOL_REG=3, RBL_REDUCE_NARROW=1), and their kernel times.
set -u
mkdir -p gpurun_out/r05_b20
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_fp32_basis.py tests/test_gpu_restarted.py \
  > gpurun_out/r05_b20/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b20/t.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r05_b20/t.log | head -20; exit $rc; }
S="--n 1250000 --steps 5 --warmup 2 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0"
REPS=3 bash tools/ab.sh r05_b20/n125 "$S" tree:RBL_CHOL_REG=3:RBL_REDUCE_NARROW=1 tree || exit 1
for v in old new; do
  if [ $v = old ]; then E="RBL_CHOL_REG=3 RBL_REDUCE_NARROW=1"; else E=""; fi
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_b20/kt_$v -o kt --output-format csv -- python3 bench.py $S > gpurun_out/r05_b20/kt_$v.log 2>&1 || exit 1
  python3 - gpurun_out/r05_b20/kt_$v $v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/kt_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "chol" in r["Name"] or "k_reduce" in r["Name"]:
        print(f"{sys.argv[2]} {r['Name'][:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.1f} us {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
done
