# SQ stall / utilisation counters for the bench kernels (one pass per counter group; no
# tracing domains).  Output: gpurun_out/sq/<pass>/s_counter_collection.csv
set -u
mkdir -p gpurun_out/sq
export TMPDIR=/tmp
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ttk"
timeout -k 10 120 rocprofv3 -L > gpurun_out/sq/counters.txt 2>&1 || true
rc=0
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS" \
           "SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/sq/p$i -o s -- $B > gpurun_out/sq/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -ne 0 ] && break
done
exit $rc
