# Round-3 A/B 10: Gram split count capped at two full waves of resident workgroups
# (RBL_G44_WAVES=2, tree) vs 3 x CUs splits for every nW (tools/variants/waves0), probe at
# n = 1e7 (one rank of C4a) and n = 1.25e6 (one of 8 ranks).  Parity tests first.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_multirank.py tests/test_gpu_fullsize.py \
  tests/test_gpu_c2_c3.py > gpurun_out/r03_ab10_tests.log 2>&1; rc=$?
echo "tree tests rc=$rc"; tail -3 gpurun_out/r03_ab10_tests.log
[ $rc -ne 0 ] && exit $rc
for n in 10000000 1250000; do
  for rep in 1 2; do
    for v in waves0 tree; do
      echo "== n=$n $v (rep $rep)"
      if [ $v = tree ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=tools/variants/$v; fi
      timeout -k 10 120 ./tools/reorth_probe $n > gpurun_out/r03_ab10_${n}_${v}_$rep.log || exit 1
      grep -E "nW= 2 |nW=18|nW=36|sum" gpurun_out/r03_ab10_${n}_${v}_$rep.log
    done
  done
done
