# Round-3 A/B 9: the Gram's LDS-DMA X staging at b = 16 (panel pairs, KC = 32: C2, C3) — tree vs
# tools/variants/g44gl0 (register staging), C2 and C3 bench lines alternating.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in g44gl0 tree; do
    if [ $v = tree ]; then unset RBL_LIB; else export RBL_LIB=$PWD/tools/variants/$v/librbl_hip.so; fi
    timeout -k 10 300 python bench.py --n 1000000 --b 16 --halfwidth 32 --steps 5 --warmup 1 \
      --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk > gpurun_out/r03_ab9_c2_${v}_$rep.json 2>/dev/null || exit 1
    timeout -k 10 300 python bench.py --matrix circuit --n 1585478 --b 16 --steps 3 --warmup 1 \
      --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk > gpurun_out/r03_ab9_c3_${v}_$rep.json 2>/dev/null || exit 1
    python - $v gpurun_out/r03_ab9_c2_${v}_$rep.json gpurun_out/r03_ab9_c3_${v}_$rep.json <<'PY'
import json, sys
for f in sys.argv[2:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    st = d["stage_ms_per_run"]
    print(f"{sys.argv[1]:6s} {d['config']['workload'][:10]:10s} value={d['value']:.2f} part_reorth={st.get('part reorth')} ms/run={d['ms_per_step']}", flush=True)
PY
  done
done
