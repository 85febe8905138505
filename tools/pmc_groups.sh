# Occupancy / LDS / MFMA counters for a command, one rocprofv3 --pmc pass per group (no
# tracing domains).  Usage: bash tools/pmc_groups.sh <outdir> <program> [args...]
# Summarise: python tools/pmc_groups_summary.py <outdir> <kernel-substring>
set -u
out=$1; shift
mkdir -p "$out"
export TMPDIR=/tmp
groups=(
 "GRBM_GUI_ACTIVE SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_LDS SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"
 "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INST_LEVEL_LDS"
 "SQ_LDS_UNALIGNED_STALL SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES"
)
# PMC_TCC=1: two more passes for the memory side (FETCH_SIZE alone takes 3 of the 4 TCC slots)
if [ "${PMC_TCC:-0}" = 1 ]; then
  groups+=("FETCH_SIZE" "WRITE_SIZE TCC_HIT_sum TCC_MISS_sum")
fi
i=0
for g in "${groups[@]}"; do
  i=$((i+1))
  timeout -k 10 600 rocprofv3 --pmc $g --output-format csv -d "$out/g$i" -o p -- "$@" > "$out/g$i.log" 2>&1
  rc=$?
  echo "group $i rc=$rc"
  [ $rc -ne 0 ] && exit $rc
done
exit 0
