# Round-3 A/B 14: the b = 16 partial-reorth update on the 32-column fast kernel
# (RBL_TSMM44_FAST32=1, no cross Gram) vs the generic kernel (default): C2 and C3 lines.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
RBL_TSMM44_FAST32=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread \
  tests/test_gpu_c2_c3.py tests/test_gpu_parity.py > gpurun_out/r03_ab14_tests.log 2>&1; rc=$?
echo "fast32 tests rc=$rc"; tail -1 gpurun_out/r03_ab14_tests.log
[ $rc -ne 0 ] && exit $rc
for rep in 1 2; do
  for f in 0 1; do
    export RBL_TSMM44_FAST32=$f
    timeout -k 10 300 python bench.py --n 1000000 --b 16 --halfwidth 32 --steps 5 --warmup 1 \
      --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk > gpurun_out/r03_ab14_c2_${f}_$rep.json 2>/dev/null || exit 1
    timeout -k 10 300 python bench.py --matrix circuit --n 1585478 --b 16 --steps 3 --warmup 1 \
      --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk > gpurun_out/r03_ab14_c3_${f}_$rep.json 2>/dev/null || exit 1
    python - $f gpurun_out/r03_ab14_c2_${f}_$rep.json gpurun_out/r03_ab14_c3_${f}_$rep.json <<'PY'
import json, sys
for f in sys.argv[2:]:
    d = json.loads(open(f).read().strip().splitlines()[-1])
    st = d["stage_ms_per_run"]
    print(f"fast32={sys.argv[1]} {d['config']['workload'][:10]:10s} value={d['value']:.2f} part_reorth={st.get('part reorth')} ms/run={d['ms_per_step']}", flush=True)
PY
  done
done
