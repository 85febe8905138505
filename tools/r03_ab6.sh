# Round-3 A/B 6: generic k_tsmm44 (b = 16 partial-reorth update, b x b applies) with hoisted Y
# addressing (tree) vs the previous commit (tools/variants/epg0): parity tests, bit identity,
# C2 (n = 1e6, b = 16) bench lines alternating.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_parity.py tests/test_gpu_golden.py tests/test_gpu_c2_c3.py tests/test_gpu_restarted.py \
  tests/test_gpu_dense.py > gpurun_out/r03_ab6_tests.log 2>&1; rc=$?
echo "tree tests rc=$rc"; tail -3 gpurun_out/r03_ab6_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/bit_tree.npz || exit 1
RBL_LIB=$PWD/tools/variants/epg0/librbl_hip.so timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/bit_epg0.npz || exit 1
python tools/r03_bitcmp.py cmp gpurun_out/bit_tree.npz gpurun_out/bit_epg0.npz
rm -f gpurun_out/bit_*.npz
for rep in 1 2; do
  for v in epg0 tree; do
    if [ $v = tree ]; then unset RBL_LIB; else export RBL_LIB=$PWD/tools/variants/$v/librbl_hip.so; fi
    timeout -k 10 300 python bench.py --n 1000000 --b 16 --halfwidth 32 --steps 5 --warmup 1 \
      --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk > gpurun_out/r03_ab6_${v}_$rep.json 2>/dev/null || exit 1
    python - $v gpurun_out/r03_ab6_${v}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st = d["stage_ms_per_run"]
print(f"{sys.argv[1]:5s} value={d['value']:.2f} ms/run part_reorth={st.get('part reorth')} loc_reorth={st.get('loc reorth')} qr={st.get('qr')}", flush=True)
PY
  done
done
