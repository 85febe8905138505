# Round-3 A/B 23: tree = B_i in LDS at b = 32 (6 waves/SIMD) vs blds8 (the same forced to 8 waves/SIMD,
# 32 registers per lane: 6 waves/SIMD (tools/variants/blds, 79 VGPRs) and 8 (blds8, 62 VGPRs
# under amdgpu_waves_per_eu(8)) vs the tree (126 VGPRs, 4).  R-MAT lines, alternating; bit check.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in tree blds8; do
    if [ $v = tree ]; then unset RBL_LIB; else export RBL_LIB=$PWD/tools/variants/$v/librbl_hip.so; fi
    timeout -k 10 300 python bench.py --matrix rmat --steps 2 --warmup 1 --rmat-steps 0 --c3-steps 0 \
      --no-cpu-baseline --no-ttk > gpurun_out/r03_ab23_rmat_${v}_$rep.json 2>/dev/null || exit 1
    for w in rmat; do
    python - $v $w gpurun_out/r03_ab23_${w}_${v}_$rep.json <<'PY'
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
RBL_LIB=$PWD/tools/variants/blds8/librbl_hip.so timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/ab23_v.npz > /dev/null || exit 1
timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/ab23_t.npz > /dev/null || exit 1
python tools/r03_bitcmp.py cmp gpurun_out/ab23_t.npz gpurun_out/ab23_v.npz
rm -f gpurun_out/ab23_*.npz
