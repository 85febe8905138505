#!/bin/bash
# round 6, batch 23: the wide-band sub-record (c4w_wideband: half-width 1024, the column
# panels) in a short default-style line, one GPU and 2 shm processes.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out/r06_b23
args="--steps 2 --warmup 1 --no-cpu-baseline --rmat-steps 0 --c3-steps 0 --c5-steps 0"
timeout -k 10 300 python bench.py $args > gpurun_out/r06_b23/one.json 2> gpurun_out/r06_b23/one.err || exit 1
timeout -k 10 400 python bench.py --gpus 2 --transport shm $args > gpurun_out/r06_b23/shm2.json 2> gpurun_out/r06_b23/shm2.err || exit 1
for f in one shm2; do
python3 - gpurun_out/r06_b23/$f.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
w = d["c4w_wideband"]
print(sys.argv[1], d["value"], "wide:", w.get("error") or (w["value"], w["roofline_secondary"]["kernel"] if w["roofline_secondary"]["kernel"].startswith("spmm") else w["roofline"]["kernel"], w["roofline_secondary"].get("ms_per_launch"), w["roofline_secondary"].get("frac"), w["time_to_k"]))
PY
done
