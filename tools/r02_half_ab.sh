# A/B of the half band tiles (default for symmetric A) against the whole tiles, and the A-load
# policy variants (RBL_BT_VAR 4099: every A load non-temporal), fuse 3 (no fused local reorth).
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "whole:RBL_BT_HALF=0" "half:RBL_BT_HALF=1" "half_nt:RBL_BT_HALF=1 RBL_BT_VAR=4099"; do
    name=${cfg%%:*}; envs=${cfg#*:}
    env $envs timeout -k 10 300 python bench.py --no-cpu-baseline --no-ttk --fuse 3 > gpurun_out/half_ab_${name}_${rep}.json 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(sys.argv[2], d['value'], d['roofline_secondary']['ms_per_launch'], d['stage_ms_per_run']['AQ'])" gpurun_out/half_ab_${name}_${rep}.json $name
  done
done
