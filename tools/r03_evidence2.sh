# Round-3 evidence 2: C5 line after keeping the automatic device-block plan across runs; PMC
# groups of the partial-reorth kernels before (8-B basis loads, tools/variants/w16off) and after
# (tree); the default bench line; its rocprofv3 kernel stats.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --n 50000000 --basis-bits 32 --keep-csr 0 --device-blocks -1 \
  --steps 1 --warmup 1 --no-cpu-baseline --no-ttk > gpurun_out/r03_bench_c5b.json 2> gpurun_out/r03_bench_c5b.err; rc=$?
echo "c5 rc=$rc"; tail -c 700 gpurun_out/r03_bench_c5b.json
[ $rc -ne 0 ] && exit $rc
LD_LIBRARY_PATH=tools/variants/w16off bash tools/pmc_groups.sh gpurun_out/r03_pmc_reorth_before ./tools/reorth_probe || exit 1
bash tools/pmc_groups.sh gpurun_out/r03_pmc_reorth_after ./tools/reorth_probe || exit 1
python tools/pmc_groups_summary.py gpurun_out/r03_pmc_reorth_before k_ > gpurun_out/r03_pmc_reorth_before.txt
python tools/pmc_groups_summary.py gpurun_out/r03_pmc_reorth_after k_ > gpurun_out/r03_pmc_reorth_after.txt
timeout -k 10 900 python bench.py > gpurun_out/r03_bench3.json 2> gpurun_out/r03_bench3.err; rc=$?
echo "bench rc=$rc"; tail -c 400 gpurun_out/r03_bench3.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03_prof_main -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-ttk --rmat-steps 1 --c3-steps 1 \
  > gpurun_out/r03_prof_main.log 2>&1; rc=$?
echo "prof rc=$rc"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python tools/r03_comm_counts.py 8 > gpurun_out/r03_comm_counts.log 2>&1; rc=$?
echo "comm counts rc=$rc"; tail -3 gpurun_out/r03_comm_counts.log | cut -c1-400
exit $rc
