#!/bin/bash
# round 5, batch 4: the b = 16 partial reorth on the real C3 / C2 lines — A/B of the update's
# 32-column fast path (RBL_TSMM44_FAST32) and the Gram's 3-chunk prefetch (variant g16pf3),
# alternating on one box; and the Gram prefetch on the probe.
set -u
mkdir -p gpurun_out/r05_b4
export TMPDIR=/tmp
for rep in 1 2; do
  for lib in tree variants/g16pf3; do
    L=""; [ "$lib" != tree ] && L="tools/$lib"
    LD_LIBRARY_PATH=$L timeout -k 10 120 tools/reorth_probe 1585478 16 72 > gpurun_out/r05_b4/probe_$(basename $lib)_$rep.log 2>&1 || exit 1
    echo "$lib rep $rep: $(tail -1 gpurun_out/r05_b4/probe_$(basename $lib)_$rep.log)"
  done
done
C3="--matrix circuit --n 1585478 --b 16 --steps 6 --warmup 1 --no-cpu-baseline --no-ttk-slow"
REPS=2 bash tools/ab.sh r05_b4/c3 "$C3" tree tree:RBL_TSMM44_FAST32=1 g16pf3 g16pf3:RBL_TSMM44_FAST32=1 || exit 1
C2="--n 1000000 --b 16 --halfwidth 32 --steps 20 --warmup 2 --no-cpu-baseline --no-ttk-slow --rmat-steps 0 --c3-steps 0"
REPS=2 bash tools/ab.sh r05_b4/c2 "$C2" tree tree:RBL_TSMM44_FAST32=1 g16pf3 g16pf3:RBL_TSMM44_FAST32=1 || exit 1
