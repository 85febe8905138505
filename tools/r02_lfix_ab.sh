# A/B of RBL_OPT_FUSE bit 2 (local reorth fused into the band-tile SpMM) on one box:
# bench lines at fuse 3 / 7 alternating (no CPU baseline, no time-to-k).
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for f in 3 7; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-ttk --fuse $f > gpurun_out/lfix_ab_${f}_${rep}.json 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print('fuse', sys.argv[2], d['value'], d['stage_ms_per_run'])" gpurun_out/lfix_ab_${f}_${rep}.json $f
  done
done
