# Round-3 A/B 24: row passes at higher occupancy (tools/variants/rg4: CholQR2's Gram-only pass
# 132 -> 126 VGPRs, 3 -> 4 waves/SIMD; the plain row update 130 -> 126, 3 -> 4) vs the tree.
# C4a and R-MAT lines alternating (qr / loc reorth stages).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in tree rg4; do
    if [ $v = tree ]; then unset RBL_LIB; else export RBL_LIB=$PWD/tools/variants/$v/librbl_hip.so; fi
    timeout -k 10 300 python bench.py --steps 3 --warmup 1 --rmat-steps 0 --c3-steps 0 \
      --no-cpu-baseline --no-ttk > gpurun_out/r03_ab24_c4a_${v}_$rep.json 2>/dev/null || exit 1
    timeout -k 10 300 python bench.py --matrix rmat --steps 2 --warmup 1 --rmat-steps 0 --c3-steps 0 \
      --no-cpu-baseline --no-ttk > gpurun_out/r03_ab24_rmat_${v}_$rep.json 2>/dev/null || exit 1
    for w in c4a rmat; do
    python - $v $w gpurun_out/r03_ab24_${w}_${v}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
st = d["stage_ms_per_run"]
print(f"{sys.argv[2]:4s} {sys.argv[1]:5s} value={d['value']:.3f} qr={st.get('qr')} 3term={st.get('3-term')} loc={st.get('loc reorth')}", flush=True)
PY
    done
  done
done
