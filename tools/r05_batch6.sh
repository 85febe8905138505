#!/bin/bash
# round 5, batch 6: the b = 16 update's 32-column fast path (RBL_TSMM44_FAST32) — compute side
# (basis aliased into cache) and the real C3 / C2 lines, alternating, 3 reps.
set -u
mkdir -p gpurun_out/r05_b6
export TMPDIR=/tmp
for f in 0 1; do
  RBL_TSMM44_FAST32=$f PROBE_W0=1 timeout -k 10 120 tools/reorth_probe 1585478 16 72 > gpurun_out/r05_b6/probe_w0_f$f.log 2>&1 || exit 1
  echo "aliased fast32=$f: $(tail -1 gpurun_out/r05_b6/probe_w0_f$f.log)"
done
C3="--matrix circuit --n 1585478 --b 16 --steps 6 --warmup 1 --no-cpu-baseline --no-ttk-slow"
REPS=3 bash tools/ab.sh r05_b6/c3 "$C3" tree tree:RBL_TSMM44_FAST32=1 || exit 1
C2="--n 1000000 --b 16 --halfwidth 32 --steps 20 --warmup 2 --no-cpu-baseline --no-ttk-slow --rmat-steps 0 --c3-steps 0"
REPS=2 bash tools/ab.sh r05_b6/c2 "$C2" tree tree:RBL_TSMM44_FAST32=1 || exit 1
