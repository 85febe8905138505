#!/bin/bash
# round 5, batch 4: the b = 16 Gram's basis prefetch.  With the X chunk staged by LDS-DMA every
# __syncthreads() drains the prefetch issued two chunks ahead (vmcnt(0)); register staging keeps
# it.  Alternating A/B on the probe (C3's shape, nW = 2..72) and on the real C3 and C2 lines:
# tree (LDS-DMA X), g16nogl (register X), g16nogl_pf3 (register X, basis 3 chunks ahead).
set -u
mkdir -p gpurun_out/r05_b4
export TMPDIR=/tmp
for rep in 1 2 3; do
  for lib in tree g16nogl g16nogl_pf3; do
    L=""; [ "$lib" != tree ] && L="$PWD/tools/variants/$lib"
    [ -n "$L" ] && [ ! -f "$L/librbl_hip.so" ] && { echo "missing $L"; exit 1; }
    LD_LIBRARY_PATH=$L timeout -k 10 120 tools/reorth_probe 1585478 16 72 > gpurun_out/r05_b4/probe_${lib}_$rep.log 2>&1 || exit 1
    echo "$lib rep $rep: $(tail -1 gpurun_out/r05_b4/probe_${lib}_$rep.log)"
  done
done
C3="--matrix circuit --n 1585478 --b 16 --steps 6 --warmup 1 --no-cpu-baseline --no-ttk-slow"
REPS=2 bash tools/ab.sh r05_b4/c3 "$C3" tree g16nogl g16nogl_pf3 || exit 1
C2="--n 1000000 --b 16 --halfwidth 32 --steps 20 --warmup 2 --no-cpu-baseline --no-ttk-slow --rmat-steps 0 --c3-steps 0"
REPS=2 bash tools/ab.sh r05_b4/c2 "$C2" tree g16nogl g16nogl_pf3 || exit 1
