# C2 (n = 1e6, b = 16) A/B on one box: update fast path on/off, local-reorth Gram fusion on/off
set -u
mkdir -p gpurun_out
for rep in 1 2; do
  for cfg in "fast1_fuse3::3" "fast1_fuse1::1" "fast0_fuse1:RBL_TSMM44_FAST=0:1"; do
    name=${cfg%%:*}; rest=${cfg#*:}; envs=${rest%%:*}; fuse=${rest##*:}
    env $envs timeout -k 10 300 python bench.py --n 1000000 --b 16 --halfwidth 32 --steps 5 --no-cpu-baseline --no-ttk --fuse $fuse > gpurun_out/c2ab_$name.json 2>&1 || exit $?
    python3 -c "import json,sys; d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][0]); print(sys.argv[2], d['value'], {k: v for k, v in d['stage_ms_per_run'].items() if v})" gpurun_out/c2ab_$name.json $name
  done
done
