#!/bin/bash
# Round-4 GPU batch: the push/pull halo split and the C5 sub-record (one gpurun call).
# Every GPU step has its own time limit; the chain stops at the first failure.
set -u
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 60 ./tools/i8_probe > gpurun_out/r04_i8_probe.log 2>&1 || echo "i8 probe rc=$?"
timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_rmat.py -k "push or ragged or without_rows" > gpurun_out/r04_push_tests.log 2>&1 &&
timeout -k 10 500 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_multiproc.py > gpurun_out/r04_push_multiproc.log 2>&1 &&
timeout -k 10 250 python -u tools/comm_counts.py 8 r04 > gpurun_out/r04_comm_counts.log 2>&1 &&
timeout -k 10 300 python bench.py --gpus 2 --transport shm --n 2000000 --steps 2 --warmup 1 \
  --rmat-steps 1 --c3-steps 1 --c5-n 8000000 > gpurun_out/r04_bench_shm2_c5.json \
  2> gpurun_out/r04_bench_shm2_c5.err &&
timeout -k 10 300 python bench.py --n 2000000 --steps 2 --rmat-steps 1 --c3-steps 1 \
  --c5-min-ranks 1 --c5-n 20000000 --no-cpu-baseline > gpurun_out/r04_bench_c5sub.json \
  2> gpurun_out/r04_bench_c5sub.err
rc=$?
echo "batch rc=$rc"
exit $rc
