# Round-3 A/B 2: update kernel k_tsmm44f with 4 row tiles per wave and KC=16
# (tools/variants/nrt4, -DRBL_T44_NRT=4 -DRBL_T44_KC=16) vs the tree (2 tiles, KC=32).
# Parity of the variant first (RBL_LIB points the Python package at it), then the probe, alternating.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
RBL_LIB=$PWD/tools/variants/nrt4/librbl_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_c5.py \
  > gpurun_out/r03_ab2_tests.log 2>&1; rc=$?
echo "variant tests rc=$rc"; tail -3 gpurun_out/r03_ab2_tests.log
[ $rc -ne 0 ] && exit $rc
REPS="1 2 3" bash tools/r02_reorth_ab.sh nrt4
