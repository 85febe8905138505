#!/bin/bash
# round 5, batch 9: the one-wave register Cholesky (k_chol_reg) — bit-identity against the
# four-wave kernel, the parity files, then the C4a / C3 lines and the kernel's own time, A/B.
set -u
mkdir -p gpurun_out/r05_b9
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  tests/test_gpu_c2_c3.py tests/test_gpu_fp32_basis.py > gpurun_out/r05_b9/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b9/t.log)"
[ $rc -ne 0 ] && exit $rc
C4="--steps 3 --warmup 1 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0"
REPS=2 bash tools/ab.sh r05_b9/c4a "$C4" tree:RBL_CHOL_REG=0 tree || exit 1
C3="--matrix circuit --n 1585478 --b 16 --steps 6 --warmup 1 --no-cpu-baseline --no-ttk-slow"
REPS=2 bash tools/ab.sh r05_b9/c3 "$C3" tree:RBL_CHOL_REG=0 tree || exit 1
for r in 0 1; do
  RBL_CHOL_REG=$r timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_b9/kt$r -o kt --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0 > gpurun_out/r05_b9/kt$r.log 2>&1 || exit 1
  python3 - gpurun_out/r05_b9/kt$r <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/kt_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "chol" in r["Name"] or "k_reduce" in r["Name"]:
        print(f"{r['Name'][:60]:60s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.1f} us {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
done
