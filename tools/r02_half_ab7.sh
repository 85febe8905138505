# Whole vs half band tiles at the default fusions (fuse 7: local reorth inside the SpMM).
set -u
mkdir -p gpurun_out
for rep in 1 2 3; do
  for h in 0 1; do
    RBL_BT_HALF=$h timeout -k 10 300 python bench.py --no-cpu-baseline --no-ttk > gpurun_out/half7_${h}_${rep}.json 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print('half', sys.argv[2], d['value'], d['roofline_secondary']['ms_per_launch'], d['stage_ms_per_run'])" gpurun_out/half7_${h}_${rep}.json $h
  done
done
