set -u
mkdir -p gpurun_out
for m in 0 1 2; do
  RBL_SPMM_ABLATE=$m timeout -k 10 300 python tools/spmm_ablate.py >> gpurun_out/ablate.log 2>&1 || exit $?
done
