# C2 / C3-shaped full-size fixture tests, then the partial-reorth kernels alone (probe) with
# timing and the PMC groups (occupancy / LDS / MFMA busy).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -v --timeout 400 --timeout-method thread \
  tests/test_gpu_c2_c3.py tests/test_gpu_memory_plan.py tests/test_gpu_fp32_basis.py > gpurun_out/r02_t2.log 2>&1; rc=$?
echo "c2/c3 tests rc=$rc"; tail -4 gpurun_out/r02_t2.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 ./tools/reorth_probe > gpurun_out/r02_reorth_probe.log 2>&1; rc=$?
echo "probe rc=$rc"; tail -3 gpurun_out/r02_reorth_probe.log
[ $rc -ne 0 ] && exit $rc
bash tools/pmc_groups.sh gpurun_out/r02_pmc_reorth ./tools/reorth_probe; rc=$?
python3 tools/pmc_groups_summary.py gpurun_out/r02_pmc_reorth 44 > gpurun_out/r02_pmc_reorth_summary.txt
cat gpurun_out/r02_pmc_reorth_summary.txt
exit $rc
