# Round-3 A/B 20: R-MAT (C4b) one-sweep segmented gather with the cold columns' Q rows loaded
# non-temporally (tools/variants/hot16k, hot128k: RBL_SEG_HOT = 16384 / 131072, hubs are the
# low ids) vs the tree (default policy everywhere).  Then the C5 test file (deep spill test).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in 1 2; do
  for v in tree hot16k hot128k; do
    if [ $v = tree ]; then unset RBL_LIB; else export RBL_LIB=$PWD/tools/variants/$v/librbl_hip.so; fi
    timeout -k 10 400 python bench.py --matrix rmat --steps 2 --warmup 1 --c3-steps 0 \
      --no-cpu-baseline --no-ttk > gpurun_out/r03_ab20_${v}_$rep.json 2>gpurun_out/r03_ab20_${v}_$rep.err || exit 1
    python - $v gpurun_out/r03_ab20_${v}_$rep.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st = d["stage_ms_per_run"]
r = d["roofline"] if "spmm" in d["roofline"]["kernel"] else d["roofline_secondary"]
print(f"{sys.argv[1]:8s} value={d['value']:.3f} AQ={st.get('AQ')} spmm_ms={r.get('ms_per_launch')}", flush=True)
PY
  done
done
unset RBL_LIB
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_c5.py \
  > gpurun_out/r03_ab20_c5.log 2>&1; rc=$?
echo "c5 tests rc=$rc"; grep -E 'PASS|FAIL|ERROR|passed|failed' gpurun_out/r03_ab20_c5.log | tail -8
exit $rc
