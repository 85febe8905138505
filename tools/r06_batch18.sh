#!/bin/bash
# round 6, batch 18: the whole -m gpu suite on the current tree (column panels v6, queue cap).
set -u
export TMPDIR=/tmp
bash tools/r06_gpu_tests.sh gpurun_out/r06_b18/tests || exit 1
