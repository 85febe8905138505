#!/bin/bash
# round 6 evidence for the default bench line: the bench JSON, then the rocprofv3 kernel-trace
# summary of the same command (PMC passes: tools/r06_final_pmc.sh, a separate call).
set -u
tag=${1:-r06_final}
mkdir -p gpurun_out/$tag
export TMPDIR=/tmp
timeout -k 10 700 python bench.py > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || exit $?
tail -c 600 gpurun_out/$tag/bench.json
timeout -k 10 700 rocprofv3 --kernel-trace --stats -d gpurun_out/$tag/prof -o run --output-format csv -- python3 bench.py \
  > gpurun_out/$tag/prof_bench.json 2> gpurun_out/$tag/prof_bench.err || exit $?
echo done
