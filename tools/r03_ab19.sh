# Round-3 A/B 19: fp64 Gram with basis panel pairs per wave (RBL_G44_DUO=1; tree build: one
# wave per SIMD, tools/variants/duo2: two, spilling) vs one panel per wave.  Bit-identity of
# the traces, the reorth probe alternating, C4a lines.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
RBL_G44_DUO=0 timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/ab19_d0.npz || exit 1
RBL_G44_DUO=1 timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/ab19_d1.npz || exit 1
python tools/r03_bitcmp.py cmp gpurun_out/ab19_d0.npz gpurun_out/ab19_d1.npz
for rep in 1 2 3; do
  for v in one duo duo2; do
    echo "== $v (rep $rep)"
    if [ $v = duo2 ]; then export LD_LIBRARY_PATH=tools/variants/duo2; else unset LD_LIBRARY_PATH; fi
    if [ $v = one ]; then export RBL_G44_DUO=0; else export RBL_G44_DUO=1; fi
    timeout -k 10 120 ./tools/reorth_probe | tail -1 || exit 1
  done
done
unset LD_LIBRARY_PATH
for rep in 1 2; do
  for v in 0 1; do
    RBL_G44_DUO=$v timeout -k 10 400 python bench.py --steps 3 --warmup 1 --rmat-steps 0 --c3-steps 0 \
      --no-cpu-baseline --no-ttk > gpurun_out/r03_ab19_${v}_$rep.json 2>/dev/null || exit 1
    python - $v gpurun_out/r03_ab19_${v}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st = d["stage_ms_per_run"]
print(f"duo={sys.argv[1]} value={d['value']:.3f} part={st.get('part reorth')}", flush=True)
PY
  done
done
