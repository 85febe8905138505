#!/bin/bash
# round 5, batch 7: per-kernel times of the C3 line with the b = 16 update on the generic kernel
# and on the 32-column fast path (RBL_TSMM44_FAST32=1): where the line's +2.5 % comes from.
set -u
mkdir -p gpurun_out/r05_b7
export TMPDIR=/tmp
C3="--matrix circuit --n 1585478 --b 16 --steps 3 --warmup 1 --no-cpu-baseline --no-ttk"
for f in 0 1; do
  RBL_TSMM44_FAST32=$f timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_b7/f$f -o kt --output-format csv -- python3 bench.py $C3 > gpurun_out/r05_b7/f$f.json 2> gpurun_out/r05_b7/f$f.err || exit 1
  python3 - gpurun_out/r05_b7/f$f <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/kt_kernel_stats.csv", recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:8]:
    print(f"{r['Name'][:64]:64s} {int(r['Calls']):5d} {float(r['AverageNs'])/1e3:9.1f} us {float(r['TotalDurationNs'])/1e6:8.1f} ms")
PY
done
