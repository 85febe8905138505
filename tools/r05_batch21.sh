#!/bin/bash
# round 5, batch 21: reduction chunks of 32 for the update's many local-reorth Gram partials
# (RBL_RED_CHUNK=0: the earlier 256 / 16) — tests touching the fused Gram, then A/Bs at the
# per-rank N = 8 size and at C4a, and the k_reduce_chunks times.
set -u
mkdir -p gpurun_out/r05_b21
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_multirank.py tests/test_gpu_spill.py > gpurun_out/r05_b21/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b21/t.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r05_b21/t.log | head -20; exit $rc; }
S="--n 1250000 --steps 5 --warmup 2 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0"
REPS=3 bash tools/ab.sh r05_b21/n125 "$S" tree:RBL_RED_CHUNK=0 tree || exit 1
C4="--steps 3 --warmup 1 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0"
REPS=2 bash tools/ab.sh r05_b21/c4a "$C4" tree:RBL_RED_CHUNK=0 tree || exit 1
for v in 0 32; do
  RBL_RED_CHUNK=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_b21/kt_$v -o kt --output-format csv -- python3 bench.py $S > gpurun_out/r05_b21/kt_$v.log 2>&1 || exit 1
  python3 - gpurun_out/r05_b21/kt_$v $v <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/kt_kernel_stats.csv", recursive=True)[0]
for r in csv.DictReader(open(f)):
    if "k_reduce" in r["Name"]:
        print(f"chunk={sys.argv[2]} {r['Name'][:55]:55s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:8.1f} us {float(r['TotalDurationNs'])/1e6:8.2f} ms")
PY
done
