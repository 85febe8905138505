# Column-tiered R-MAT SpMM A/B (C4b: n = 1e7, scale 24, b = 32): AQ ms per launch for each
# RBL_SEG_TIERS setting, alternating, two rounds; then rocprofv3 kernel stats of the best guess.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for round in 1 2; do
  for t in none 16384 8192 16384,262144 16384,1048576 4096,65536; do
    if [ "$t" = none ]; then unset RBL_SEG_TIERS; else export RBL_SEG_TIERS=$t; fi
    timeout -k 10 300 python bench.py --matrix rmat --steps 2 --warmup 1 --no-cpu-baseline --no-ttk \
      > gpurun_out/r03_tiers_${t}_${round}.json 2> gpurun_out/r03_tiers_${t}_${round}.err || exit 1
    python - "$t" gpurun_out/r03_tiers_${t}_${round}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"] if "spmm" in d["roofline"]["kernel"] else d["roofline_secondary"]
print(f"tiers={sys.argv[1]:>14} value={d['value']:.3f} AQ ms/launch={r['ms_per_launch']:.3f} "
      f"stage AQ={d['stage_ms_per_run']['AQ']:.1f}", flush=True)
PY
  done
done
unset RBL_SEG_TIERS
export RBL_SEG_TIERS=16384,262144
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/r03_prof_tiers -o run -- \
  python bench.py --matrix rmat --steps 1 --warmup 0 --no-cpu-baseline --no-ttk \
  > gpurun_out/r03_prof_tiers.log 2>&1 || exit 1
find gpurun_out/r03_prof_tiers -name "*kernel_stats.csv" | head -3
