# Round-3 A/B 26: segmented gather with a row pipeline (tools/variants/rpf: the bounds of row
# rr + 2R and the first chunk of row rr + R load before row rr's gathers; b = 32 84 VGPRs / 5
# waves, b = 16 116 / 4; rpfw: the same held to 6 / 5 waves, a few spills) vs the tree (b = 32:
# 64 VGPRs / 8 waves, b = 16: 94 / 5).  C3-shape and R-MAT lines alternating; bit check.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in tree rpf rpfw; do
    if [ $v = tree ]; then unset RBL_LIB; else export RBL_LIB=$PWD/tools/variants/$v/librbl_hip.so; fi
    timeout -k 10 300 python bench.py --matrix circuit --n 1585478 --b 16 --k 20 --steps 5 --warmup 1 \
      --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk > gpurun_out/r03_ab26_c3_${v}_$rep.json 2>/dev/null || exit 1
    timeout -k 10 300 python bench.py --matrix rmat --steps 2 --warmup 1 --rmat-steps 0 --c3-steps 0 \
      --no-cpu-baseline --no-ttk > gpurun_out/r03_ab26_rmat_${v}_$rep.json 2>/dev/null || exit 1
    for w in c3 rmat; do
    python - $v $w gpurun_out/r03_ab26_${w}_${v}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
st = d["stage_ms_per_run"]
r = d["roofline"] if "spmm" in d["roofline"]["kernel"] else d["roofline_secondary"]
print(f"{sys.argv[2]:4s} {sys.argv[1]:5s} value={d['value']:.3f} AQ={st.get('AQ')} spmm_ms={r.get('ms_per_launch')}", flush=True)
PY
    done
  done
done
unset RBL_LIB
RBL_LIB=$PWD/tools/variants/rpf/librbl_hip.so timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/ab26_v.npz > /dev/null || exit 1
timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/ab26_t.npz > /dev/null || exit 1
python tools/r03_bitcmp.py cmp gpurun_out/ab26_t.npz gpurun_out/ab26_v.npz
rm -f gpurun_out/ab26_*.npz
