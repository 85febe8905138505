#!/bin/bash
# round 5, batch 18: same-box A/B on the headline (C4a), this morning's library (HEAD at the
# start of the session's latency work, tools/variants/head) against the tree
set -u
mkdir -p gpurun_out/r05_b18
export TMPDIR=/tmp
C4="--steps 3 --warmup 1 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0"
REPS=3 bash tools/ab.sh r05_b18/c4a "$C4" head tree || exit 1
