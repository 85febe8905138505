# Round-3 evidence 1: C5 wall-time attribution (bench line + rocprofv3 kernel/memory-copy
# trace), R-MAT column-tier PMC counters (L2 hit rate, fabric bytes per k_spmm_seg launch), the
# C2 line with AI-based pricing, the C3-shaped circuit line + its kernel stats.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
B1="--steps 1 --warmup 0 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0"
# R-MAT tiers: TCC hit / miss and FETCH_SIZE of the seg kernel launches, one pass per group
for t in none 4096,65536; do
  if [ "$t" = none ]; then unset RBL_SEG_TIERS; else export RBL_SEG_TIERS=$t; fi
  i=0
  for g in "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
    i=$((i+1))
    timeout -s KILL 240 rocprofv3 --pmc $g --kernel-include-regex k_spmm_seg --output-format csv \
      -d gpurun_out/r03_pmc_tiers/$t/g$i -o p -- python3 bench.py --matrix rmat $B1 \
      > gpurun_out/r03_pmc_tiers_${t}_g$i.log 2>&1 || { echo "pmc $t g$i failed"; exit 1; }
  done
done
unset RBL_SEG_TIERS
echo "pmc tiers done"
timeout -k 10 300 python bench.py --n 1000000 --b 16 --halfwidth 32 --steps 5 --warmup 1 \
  --rmat-steps 0 --c3-steps 0 --no-cpu-baseline > gpurun_out/r03_bench_c2.json 2> gpurun_out/r03_bench_c2.err || exit 1
echo "c2 done"; tail -c 600 gpurun_out/r03_bench_c2.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_prof_c3 -o run -- \
  python3 bench.py --matrix circuit --n 1585478 --b 16 --steps 3 --warmup 1 --rmat-steps 0 --c3-steps 0 \
  --no-cpu-baseline > gpurun_out/r03_bench_c3.json 2> gpurun_out/r03_bench_c3.err || exit 1
echo "c3 done"; tail -c 600 gpurun_out/r03_bench_c3.json
bash tools/r03_c5_diag.sh
