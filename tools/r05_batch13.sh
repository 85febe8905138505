#!/bin/bash
# round 5, batch 13: the elimination Cholesky (RBL_CHOL_REG=2) — tests, then the per-rank N = 8
# C4a size and the full C4a line against the register kernel (1), alternating; kernel times.
# The whole -m gpu suite first: the tree also carries the fused end-of-step stash (k_stash).
set -u
mkdir -p gpurun_out/r05_b13
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread tests \
  > gpurun_out/r05_b13/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b13/t.log)"
[ $rc -ne 0 ] && exit $rc
S="--n 1250000 --steps 5 --warmup 2 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0"
REPS=3 bash tools/ab.sh r05_b13/n125 "$S" tree:RBL_CHOL_REG=1 tree:RBL_CHOL_REG=2 || exit 1
C4="--steps 3 --warmup 1 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0"
REPS=1 bash tools/ab.sh r05_b13/c4a "$C4" tree:RBL_CHOL_REG=1 tree:RBL_CHOL_REG=2 || exit 1
for r in 1 2; do
  RBL_CHOL_REG=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_b13/kt$r -o kt --output-format csv -- python3 bench.py $S > gpurun_out/r05_b13/kt$r.log 2>&1 || exit 1
  python3 - gpurun_out/r05_b13/kt$r <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/kt_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "chol" in r["Name"]:
        print(f"{r['Name'][:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.1f} us {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
done
