# Round-3 A/B 25: segmented gather with the next chunk's col/val prefetched (tools/variants/pf:
# 87 VGPRs, 5 waves/SIMD; pf6: the same held to 6 waves) vs the tree (79 VGPRs, 6 waves).
# R-MAT lines alternating; bit check (pf6 vs tree).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in tree pf pf6; do
    if [ $v = tree ]; then unset RBL_LIB; else export RBL_LIB=$PWD/tools/variants/$v/librbl_hip.so; fi
    timeout -k 10 300 python bench.py --matrix rmat --steps 2 --warmup 1 --rmat-steps 0 --c3-steps 0 \
      --no-cpu-baseline --no-ttk > gpurun_out/r03_ab25_rmat_${v}_$rep.json 2>/dev/null || exit 1
    for w in rmat; do
    python - $v $w gpurun_out/r03_ab25_${w}_${v}_$rep.json <<'PY'
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
RBL_LIB=$PWD/tools/variants/pf6/librbl_hip.so timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/ab25_v.npz > /dev/null || exit 1
timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/ab25_t.npz > /dev/null || exit 1
python tools/r03_bitcmp.py cmp gpurun_out/ab25_t.npz gpurun_out/ab25_v.npz
rm -f gpurun_out/ab25_*.npz
