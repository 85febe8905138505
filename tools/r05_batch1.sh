#!/bin/bash
# round 5, first GPU batch: the changed tests (P = 3 / 8 over RCCL, the path counters, the push
# allocation vote), then one default bench line (CPU cross-check measured in the run).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -v --timeout 400 --timeout-method thread \
  tests/test_gpu_multirank.py::test_multirank_fused_local_reorth_runs \
  tests/test_gpu_rmat.py::test_push_buffer_allocation_failure_is_collective \
  tests/test_gpu_multiproc.py -k "rccl or fused_local_reorth_runs or push_buffer_allocation" > gpurun_out/r05_t1.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -5 gpurun_out/r05_t1.log
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py --steps 3 > gpurun_out/r05_b1.json 2> gpurun_out/r05_b1.err; rc=$?
echo "bench rc=$rc"; tail -c 1500 gpurun_out/r05_b1.json
exit $rc
