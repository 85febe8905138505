#!/bin/bash
# round 6, batch 27: LDS reads two groups ahead for <8, 16> (tools/variants/ra2, -DRBL_PANEL_RA=2)
# against the product (one group ahead) — the panel tests on the variant first, then alternating
# sweeps at H = 1024 and 2048 (the half-widths that take <8, 16>).
set -u
mkdir -p gpurun_out/r06_b27
export TMPDIR=/tmp
RBL_LIB=tools/variants/ra2/librbl_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_spmm.py tests/test_gpu_multirank.py \
  -m gpu -x -v --timeout 200 --timeout-method thread -k "panel" > gpurun_out/r06_b27/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r06_b27/pytest.log
[ $rc -ne 0 ] && { grep -E "Error|assert" gpurun_out/r06_b27/pytest.log | head; exit $rc; }
for rep in 1 2; do
  echo "== product (one group ahead), rep $rep"
  bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b27/p$rep 1024 2048 || exit 1
  echo "== ra2 (two groups ahead), rep $rep"
  RBL_LIB=tools/variants/ra2/librbl_hip.so bash tools/r06_halfwidth_sweep.sh gpurun_out/r06_b27/r$rep 1024 2048 || exit 1
done
