# Round-3 A/B 3: LDS-DMA staging (global_load_lds_dwordx4) of the X chunk in k_gram44 and the
# C chunk in k_tsmm44f (tree: RBL_G44_GLDS = RBL_T44_GLDS = 1) vs register staging
# (tools/variants/gl0).  Tree parity tests, bit identity tree vs variant, then the probe.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_c5.py tests/test_gpu_spill.py \
  tests/test_gpu_fullsize.py tests/test_gpu_multirank.py > gpurun_out/r03_ab3_tests.log 2>&1; rc=$?
echo "tree tests rc=$rc"; tail -3 gpurun_out/r03_ab3_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/bit_tree.npz || exit 1
RBL_LIB=$PWD/tools/variants/gl0/librbl_hip.so timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/bit_gl0.npz || exit 1
python tools/r03_bitcmp.py cmp gpurun_out/bit_tree.npz gpurun_out/bit_gl0.npz
REPS="1 2 3" bash tools/r02_reorth_ab.sh gl0
