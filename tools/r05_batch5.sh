#!/bin/bash
# round 5, batch 5: the basis access patterns without MFMA work (basis_stream_probe), the shipped
# kernels with the basis aliased into cache (PROBE_W0=1), and the interleaved-split Gram
# (RBL_G44_INTER16 / RBL_G44_INTER): probe and line A/Bs plus the parity tests on the variant.
set -u
mkdir -p gpurun_out/r05_b5
export TMPDIR=/tmp
timeout -k 10 180 tools/basis_stream_probe 1585478 72 > gpurun_out/r05_b5/stream.log 2>&1; rc=$?
cat gpurun_out/r05_b5/stream.log
[ $rc -ne 0 ] && exit $rc
PROBE_W0=1 timeout -k 10 120 tools/reorth_probe 1585478 16 72 > gpurun_out/r05_b5/probe_w0.log 2>&1 || exit 1
echo "aliased: $(tail -1 gpurun_out/r05_b5/probe_w0.log)"
for rep in 1 2 3; do
  for lib in tree g16inter; do
    L=""; [ "$lib" != tree ] && L="$PWD/tools/variants/$lib"
    LD_LIBRARY_PATH=$L timeout -k 10 120 tools/reorth_probe 1585478 16 72 > gpurun_out/r05_b5/probe_${lib}_$rep.log 2>&1 || exit 1
    echo "$lib rep $rep: $(tail -1 gpurun_out/r05_b5/probe_${lib}_$rep.log)"
  done
done
RBL_LIB=$PWD/tools/variants/ginter/librbl_hip.so timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread tests/test_gpu_c2_c3.py tests/test_gpu_parity.py > gpurun_out/r05_b5/t_ginter.log 2>&1; rc=$?
echo "parity on ginter rc=$rc: $(tail -1 gpurun_out/r05_b5/t_ginter.log)"
[ $rc -ne 0 ] && exit $rc
C3="--matrix circuit --n 1585478 --b 16 --steps 6 --warmup 1 --no-cpu-baseline --no-ttk-slow"
REPS=2 bash tools/ab.sh r05_b5/c3 "$C3" tree g16inter || exit 1
C4="--steps 3 --warmup 1 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0"
REPS=2 bash tools/ab.sh r05_b5/c4a "$C4" tree ginter || exit 1
