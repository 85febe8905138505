# Round-3 A/B 1: (a) Gram 16-B basis loads (RBL_G44_W16, tree) vs 8-B (tools/variants/w16off)
# with the partial-reorth probe, alternating; (b) R-MAT SpMM: persistent seg kernel with 16
# gathers in flight (RBL_SEG_V=1, default) vs the one-task-per-wave kernel (RBL_SEG_V=0);
# (c) tests that exercise both.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_spmm.py tests/test_gpu_rmat.py tests/test_gpu_parity.py \
  > gpurun_out/r03_ab1_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 gpurun_out/r03_ab1_tests.log
[ $rc -ne 0 ] && exit $rc
REPS="1 2" bash tools/r02_reorth_ab.sh w16off > gpurun_out/r03_ab1_reorth.log 2>&1 || exit 1
cat gpurun_out/r03_ab1_reorth.log
for round in 1 2; do
  for v in 0 1; do
    RBL_SEG_V=$v timeout -k 10 300 python bench.py --matrix rmat --steps 2 --warmup 1 --no-cpu-baseline --no-ttk \
      > gpurun_out/r03_segv${v}_${round}.json 2> gpurun_out/r03_segv${v}_${round}.err || exit 1
    python - "$v" gpurun_out/r03_segv${v}_${round}.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
r = d["roofline"] if "spmm" in d["roofline"]["kernel"] else d["roofline_secondary"]
print(f"segv={sys.argv[1]} value={d['value']:.3f} AQ ms/launch={r['ms_per_launch']:.3f} "
      f"gather GB/s={r.get('gbs_incl_q_row_gathers')}", flush=True)
PY
  done
done
