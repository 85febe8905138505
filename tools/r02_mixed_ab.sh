# A/B of the fp32-basis (mixed) bench: tools/variants/<name>/librbl_hip.so vs the tree, alternating
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "$@" tree; do
    if [ "$v" = tree ]; then lib=""; else lib="RBL_LIB=tools/variants/$v/librbl_hip.so"; fi
    env $lib timeout -k 10 300 python bench.py --basis-bits 32 --no-cpu-baseline --no-ttk > gpurun_out/mixab_$v.json 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(sys.argv[2], d['value'], d['stage_ms_per_run']['part reorth'])" gpurun_out/mixab_$v.json $v
  done
done
