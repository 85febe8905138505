#!/bin/bash
# round 6, batch 28: the fp32 Gram (k_gram32x) in 64-row chunks (tools/variants/g64,
# -DRBL_G32X_ROWS=64: half the barriers per basis row) against the shipped 32 — the fp32-basis
# tests on the variant first, then the fp32 C4a line (partial reorth) alternating.
set -u
mkdir -p gpurun_out/r06_b28
export TMPDIR=/tmp
RBL_LIB=tools/variants/g64/librbl_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fp32_basis.py \
  -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r06_b28/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/r06_b28/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06_b28/pytest.log | head; exit $rc; }
args="--basis-bits 32 --steps 3 --warmup 1 --rmat-steps 0 --c3-steps 0 --wide-steps 0 --no-cpu-baseline --no-ttk"
for rep in 1 2; do
  for v in product g64; do
    if [ $v = g64 ]; then export RBL_LIB=tools/variants/g64/librbl_hip.so; else unset RBL_LIB; fi
    timeout -k 10 300 python bench.py $args > gpurun_out/r06_b28/$v$rep.json 2> gpurun_out/r06_b28/$v$rep.err || exit 1
    python3 - gpurun_out/r06_b28/$v$rep.json $v $rep <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]
print(f"{sys.argv[2]:8s} rep {sys.argv[3]}: {d['value']} block-iters/s, partial reorth {r['ms_per_run']} ms/run = {r['frac']} of fp32 peak", flush=True)
PY
  done
done
