# Round-3 A/B 13: loads/stores as a uniform base + unsigned 32-bit lane offset in the update
# kernel (loop VALU 24 -> 10 per 256 MFMAs), the Gram's basis loads and the fused row ops
# (uniform partial-block handling) — tree vs the previous commit (tools/variants/addr0).
# Parity tests, bit identity, probe and C4a bench lines alternating.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_fp32_basis.py tests/test_gpu_multirank.py \
  tests/test_gpu_c2_c3.py tests/test_gpu_spill.py > gpurun_out/r03_ab13_tests.log 2>&1; rc=$?
echo "tree tests rc=$rc"; tail -2 gpurun_out/r03_ab13_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/bit_tree.npz || exit 1
RBL_LIB=$PWD/tools/variants/addr0/librbl_hip.so timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/bit_addr0.npz || exit 1
python tools/r03_bitcmp.py cmp gpurun_out/bit_tree.npz gpurun_out/bit_addr0.npz
rm -f gpurun_out/bit_*.npz
REPS="1 2 3" bash tools/r02_reorth_ab.sh addr0
for rep in 1 2; do
  for v in addr0 tree; do
    if [ $v = tree ]; then unset RBL_LIB; else export RBL_LIB=$PWD/tools/variants/$v/librbl_hip.so; fi
    timeout -k 10 400 python bench.py --steps 3 --warmup 1 --rmat-steps 0 --c3-steps 0 --no-cpu-baseline \
      --no-ttk > gpurun_out/r03_ab13_${v}_$rep.json 2>/dev/null || exit 1
    python - $v gpurun_out/r03_ab13_${v}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st = d["stage_ms_per_run"]
print(f"{sys.argv[1]:5s} value={d['value']:.3f} ms/run={d['ms_per_step']} qr={st.get('qr')} 3-term={st.get('3-term')} part={st.get('part reorth')} AQ={st.get('AQ')}", flush=True)
PY
  done
done
