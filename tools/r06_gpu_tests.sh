#!/bin/bash
# round 6: the -m gpu suite on the box (log under gpurun_out/<dir>), optional pytest args after
# the directory.  Usage: tools/r06_gpu_tests.sh <outdir> [pytest args...]
set -u
out=${1:-gpurun_out/r06_tests}; shift
mkdir -p $out
export TMPDIR=/tmp
timeout -k 20 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "$@" \
  > $out/pytest.log 2>&1; rc=$?
tail -5 $out/pytest.log
grep -E "FAILED|Error" $out/pytest.log | head -20
exit $rc
