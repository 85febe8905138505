# A/B of RBL_OPT_FUSE on one box: bench lines at fuse 0 / 3 alternating (no CPU baseline).
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for f in 0 3; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --no-ttk --fuse $f > gpurun_out/fuse_ab_${f}_${rep}.json 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print('fuse', sys.argv[2], d['value'], d['stage_ms_per_run'])" gpurun_out/fuse_ab_${f}_${rep}.json $f
  done
done
