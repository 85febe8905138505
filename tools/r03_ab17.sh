# Round-3 A/B 17: fp32 Gram on v_mfma_f32_32x32x2f32 (tree, k_gram32x) vs 16x16x4f32
# (tools/variants/mf16).  fp32 tests, fp32 probe alternating, C4a mixed-mode lines.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_fp32_basis.py tests/test_gpu_c5.py tests/test_gpu_spill.py > gpurun_out/r03_ab17_tests.log 2>&1; rc=$?
echo "tree tests rc=$rc"; tail -1 gpurun_out/r03_ab17_tests.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2 3; do
  for v in mf16 tree; do
    echo "== $v (rep $rep)"
    if [ $v = tree ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=tools/variants/$v; fi
    timeout -k 10 120 ./tools/reorth32_probe | tail -1 || exit 1
  done
done
unset LD_LIBRARY_PATH
for rep in 1 2; do
  for v in mf16 tree; do
    if [ $v = tree ]; then unset RBL_LIB; else export RBL_LIB=$PWD/tools/variants/$v/librbl_hip.so; fi
    timeout -k 10 400 python bench.py --basis-bits 32 --steps 3 --warmup 1 --rmat-steps 0 --c3-steps 0 \
      --no-cpu-baseline --no-ttk > gpurun_out/r03_ab17_${v}_$rep.json 2>/dev/null || exit 1
    python - $v gpurun_out/r03_ab17_${v}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st = d["stage_ms_per_run"]
print(f"{sys.argv[1]:6s} value={d['value']:.3f} part={st.get('part reorth')} loc={st.get('loc reorth')}", flush=True)
PY
  done
done
