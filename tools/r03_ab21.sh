# Round-3 A/B 21: b = 16 Gram (panel pairs) at 4 waves per SIMD (tools/variants/g4:
# RBL_G44_WPE16=4, 106 VGPRs, splits 4 x CUs) vs 3 (tree).  Probe at C3's and C2's n, then
# C3-shape and C2 bench lines.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2 3; do
  for v in tree g4; do
    if [ $v = tree ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=tools/variants/$v; fi
    echo "== $v (rep $rep) C3: $(timeout -k 10 120 ./tools/reorth_probe 1585478 16 72 | tail -1)"
    echo "== $v (rep $rep) C2: $(timeout -k 10 120 ./tools/reorth_probe 1000000 16 74 | tail -1)"
  done
done
unset LD_LIBRARY_PATH
for rep in 1 2; do
  for v in tree g4; do
    if [ $v = tree ]; then unset RBL_LIB; else export RBL_LIB=$PWD/tools/variants/$v/librbl_hip.so; fi
    timeout -k 10 300 python bench.py --matrix circuit --n 1585478 --b 16 --k 20 --steps 5 --warmup 1 \
      --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk > gpurun_out/r03_ab21_c3_${v}_$rep.json 2>/dev/null || exit 1
    timeout -k 10 300 python bench.py --n 1000000 --b 16 --halfwidth 32 --steps 5 --warmup 1 \
      --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk > gpurun_out/r03_ab21_c2_${v}_$rep.json 2>/dev/null || exit 1
    for w in c3 c2; do
    python - $v $w gpurun_out/r03_ab21_${w}_${v}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
st = d["stage_ms_per_run"]
print(f"{sys.argv[2]} {sys.argv[1]:5s} value={d['value']:.3f} part={st.get('part reorth')}", flush=True)
PY
    done
  done
done
