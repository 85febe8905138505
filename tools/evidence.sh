# Bench lines for every workload the repo claims numbers for (C4a fp64 / fp32 basis, C4b R-MAT,
# C2, host spill); each to gpurun_out/ev_<name>.json.  Usage: bash tools/evidence.sh
set -u
mkdir -p gpurun_out
run() {
  name=$1; shift
  timeout -k 10 600 python bench.py "$@" > gpurun_out/ev_$name.json 2> gpurun_out/ev_$name.err || exit $?
  echo "$name: $(python3 -c "import json;d=json.load(open('gpurun_out/ev_$name.json'));print(d['value'], d['unit'])")"
}
run c4a_fp64 --steps 3 --no-cpu-baseline
run c4a_fp32 --basis-bits 32 --steps 3 --no-cpu-baseline
run c4b_rmat --matrix rmat --steps 2 --no-cpu-baseline
run c2_b16 --n 1000000 --b 16 --halfwidth 32 --steps 5 --no-cpu-baseline
run c4a_spill20 --device-blocks 20 --steps 1 --no-cpu-baseline --no-ttk
