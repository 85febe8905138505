#!/bin/bash
# round 5, third GPU batch: C4a against the full-size oracle fixture, the push split's entry-hash
# symmetry check (R-MAT tests, shm processes), the b = 16 update A/B (generic k_tsmm44 against
# the 32-column fast path), then the N = 8 RCCL rehearsal of the bench (progress on stderr).
set -u
mkdir -p gpurun_out/r05_b3
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread \
  tests/test_gpu_fullsize.py::test_c4a_full_size_vs_oracle tests/test_gpu_rmat.py \
  > gpurun_out/r05_b3/t_a.log 2>&1; rc=$?
echo "pytest a rc=$rc"; tail -3 gpurun_out/r05_b3/t_a.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u -m pytest -v --timeout 400 --timeout-method thread \
  tests/test_gpu_multiproc.py -k "not rccl" > gpurun_out/r05_b3/t_b.log 2>&1; rc=$?
echo "pytest b rc=$rc"; tail -3 gpurun_out/r05_b3/t_b.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for f in 0 1; do
    RBL_TSMM44_FAST32=$f timeout -k 10 120 tools/reorth_probe 1585478 16 72 > gpurun_out/r05_b3/probe_f${f}_$rep.log 2>&1 || exit 1
    echo "fast32=$f rep $rep: $(tail -1 gpurun_out/r05_b3/probe_f${f}_$rep.log)"
  done
done
RBL_TSMM44_FAST32=1 PMC_TCC=1 bash tools/pmc_groups.sh gpurun_out/r05_b3/pmc_f1 tools/reorth_probe 1585478 16 72 || exit 1
python3 tools/pmc_groups_summary.py gpurun_out/r05_b3/pmc_f1 tsmm > gpurun_out/r05_b3/pmc_f1_summary.txt 2>&1
cat gpurun_out/r05_b3/pmc_f1_summary.txt
RBL_RCCL_HOST_PER_RANK=1 NCCL_DEBUG=WARN timeout -k 20 800 python bench.py --gpus 8 --n 2000000 \
  --steps 2 --warmup 1 --rmat-steps 1 --rmat-as-drawn-steps 0 --c3-steps 1 --no-ttk-slow \
  --c5-n 8000000 --c5-steps 1 > gpurun_out/r05_bench_rccl8.json 2> gpurun_out/r05_bench_rccl8.err; rc=$?
echo "rccl8 bench rc=$rc"; grep "^\[bench" gpurun_out/r05_bench_rccl8.err | tail -5; tail -c 400 gpurun_out/r05_bench_rccl8.json
exit $rc
