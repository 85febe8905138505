# SpMM ablations (RBL_SPMM_ABLATE, read once per process): one mode per process.
set -u
mkdir -p gpurun_out
for m in ${MODES:-0 1 2 3}; do
  RBL_SPMM_PROF=${PROF:-0} RBL_SPMM_ABLATE=$m timeout -k 10 300 python tools/spmm_ablate.py >> gpurun_out/ablate.log 2>&1 || exit $?
done
