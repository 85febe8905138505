#!/bin/bash
# round 6, batch 20: same-box A/B of the C4a line, the round-5 final tree (2f3f2ea, built from
# git into tools/variants/r05tree) against this tree, alternating, C4a runs only.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_b20
args="--steps 10 --warmup 3 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0 --c5-steps 0"
for i in 1 2 3; do
  for t in r05 r06; do
    if [ $t = r05 ]; then d=tools/variants/r05tree; else d=.; fi
    (cd $d && timeout -k 10 300 python bench.py $args) > gpurun_out/r06_b20/${t}_$i.json 2> gpurun_out/r06_b20/${t}_$i.err || exit 1
    python3 - gpurun_out/r06_b20/${t}_$i.json $t $i <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[2], sys.argv[3], d["value"], "reorth", d["roofline"]["ms_per_run"], "spmm", d["roofline_secondary"]["ms_per_launch"], d["stage_ms_per_run"])
PY
  done
done
