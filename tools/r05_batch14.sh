#!/bin/bash
# round 5, batch 14: k_stash writing the step record into coherent pinned memory (no D2H copy),
# the elimination Cholesky as default, the bench's timed pass without stage timers.
# The whole -m gpu suite; then an A/B at the per-rank N = 8 size (HEAD library / copy path /
# direct); a kernel trace of the direct path for the inter-kernel gaps; the default line.
set -u
mkdir -p gpurun_out/r05_b14
export TMPDIR=/tmp
timeout -k 10 560 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread tests \
  > gpurun_out/r05_b14/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b14/t.log)"
[ $rc -ne 0 ] && exit $rc
S="--n 1250000 --steps 5 --warmup 2 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0"
REPS=2 bash tools/ab.sh r05_b14/n125 "$S" head:RBL_CHOL_REG=2 tree:RBL_STASH_COPY=1 tree || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r05_b14/kt -o kt --output-format csv -- python3 bench.py $S > gpurun_out/r05_b14/kt.log 2>&1 || exit 1
timeout -k 10 600 python bench.py --no-cpu-baseline > gpurun_out/r05_b14/bench.json 2> gpurun_out/r05_b14/bench.err || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/r05_b14/bench.json').read().strip().splitlines()[-1])
print('default', d['value'], d['ms_per_step'], d['stage_pass_ms_per_run'], d['roofline']['frac'], d['roofline_secondary']['frac'])"
