# Round-3 A/B 5: k_tsmm44f epilogue with hoisted Y addressing (tree) vs the per-store division /
# 64-bit multiply form (tools/variants/ep0 = the previous commit).  Parity tests, bit identity, probe.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_c5.py tests/test_gpu_spill.py \
  tests/test_gpu_fullsize.py tests/test_gpu_multirank.py tests/test_gpu_c2_c3.py > gpurun_out/r03_ab5_tests.log 2>&1; rc=$?
echo "tree tests rc=$rc"; tail -3 gpurun_out/r03_ab5_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/bit_tree.npz || exit 1
RBL_LIB=$PWD/tools/variants/ep0/librbl_hip.so timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/bit_ep0.npz || exit 1
python tools/r03_bitcmp.py cmp gpurun_out/bit_tree.npz gpurun_out/bit_ep0.npz
rm -f gpurun_out/bit_*.npz
REPS="1 2 3" bash tools/r02_reorth_ab.sh ep0
