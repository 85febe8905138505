# Band-tile SpMM tuning variants (RBL_BT_VAR, read once per process): one variant per process,
# AQ stage ms per launch at C4a over an 8-step Lanczos run (tools/spmm_ablate.py).
set -u
mkdir -p gpurun_out
for v in ${VARS:-3 0 35}; do
  echo -n "var $v: " >> gpurun_out/bt_tune.log
  RBL_BT_VAR=$v timeout -k 10 120 python tools/spmm_ablate.py >> gpurun_out/bt_tune.log 2>&1 || exit $?
done
cat gpurun_out/bt_tune.log
