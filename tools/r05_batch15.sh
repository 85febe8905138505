#!/bin/bash
# round 5, batch 15: CholQR's pass-3 Gram and the next step's local-reorth Gram in one
# all-reduce (k_cloc_rinv after a shifted third pass); R1^-1 written by the first Cholesky
# straight into its slot.  The shift probe, the whole -m gpu suite, then the collectives per
# block step at P = 8 in-process ranks, this tree against the HEAD library.
set -u
mkdir -p gpurun_out/r05_b15
export TMPDIR=/tmp
timeout -k 10 120 python -u tools/r05_shift_probe.py > gpurun_out/r05_b15/shift.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/r05_b15/shift.log; exit 1; }
cat gpurun_out/r05_b15/shift.log
timeout -k 10 560 python -u -m pytest -v -m gpu --timeout 200 --timeout-method thread tests \
  > gpurun_out/r05_b15/t.log 2>&1; rc=$?
echo "tests rc=$rc: $(tail -1 gpurun_out/r05_b15/t.log)"
[ $rc -ne 0 ] && { grep -E "FAILED|Error" gpurun_out/r05_b15/t.log | head -20; exit $rc; }
timeout -k 10 300 python -u tools/comm_counts.py 8 r05_b15_tree > gpurun_out/r05_b15/cc_tree.log 2>&1 || exit 1
RBL_LIB=$PWD/tools/variants/head/librbl_hip.so timeout -k 10 300 python -u tools/comm_counts.py 8 r05_b15_head > gpurun_out/r05_b15/cc_head.log 2>&1 || exit 1
grep -o '^[^{]*\|"allreduce_calls": \[[^]]*\]' gpurun_out/r05_b15/cc_head.log gpurun_out/r05_b15/cc_tree.log
S="--n 1250000 --steps 5 --warmup 2 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0"
REPS=2 bash tools/ab.sh r05_b15/n125 "$S" head:RBL_CHOL_REG=2 tree || exit 1
