# Round-3 A/B 7: CholQR applies on the triangular R^-1 skip the all-zero MFMA blocks
# (k_rowgram TRI, tree) vs every block multiplied (tools/variants/tri0 = previous commit).
# Parity tests, bit identity of short runs, C4a bench lines alternating (qr stage).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_c5.py tests/test_gpu_spill.py \
  tests/test_gpu_fullsize.py tests/test_gpu_multirank.py tests/test_gpu_c2_c3.py tests/test_gpu_fp32_basis.py \
  tests/test_gpu_restarted.py > gpurun_out/r03_ab7_tests.log 2>&1; rc=$?
echo "tree tests rc=$rc"; tail -3 gpurun_out/r03_ab7_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/bit_tree.npz || exit 1
RBL_LIB=$PWD/tools/variants/tri0/librbl_hip.so timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/bit_tri0.npz || exit 1
python tools/r03_bitcmp.py cmp gpurun_out/bit_tree.npz gpurun_out/bit_tri0.npz
rm -f gpurun_out/bit_*.npz
for rep in 1 2; do
  for v in tri0 tree; do
    if [ $v = tree ]; then unset RBL_LIB; else export RBL_LIB=$PWD/tools/variants/$v/librbl_hip.so; fi
    timeout -k 10 400 python bench.py --steps 3 --warmup 1 --rmat-steps 0 --c3-steps 0 --no-cpu-baseline \
      --no-ttk > gpurun_out/r03_ab7_${v}_$rep.json 2>/dev/null || exit 1
    python - $v gpurun_out/r03_ab7_${v}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st = d["stage_ms_per_run"]
print(f"{sys.argv[1]:5s} value={d['value']:.3f} ms/run={d['ms_per_step']} qr={st.get('qr')} 3-term={st.get('3-term')} part={st.get('part reorth')} AQ={st.get('AQ')}", flush=True)
PY
  done
done
