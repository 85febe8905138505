# C5 (n = 5e7, fp32 basis, one GPU, host spill) wall-time attribution: one timed run under
# rocprofv3 kernel + memory-copy trace (no counters), then the same bench line without the
# profiler (stage times incl. the new "spill wait" stage, host_ms_per_run).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python bench.py --n 50000000 --basis-bits 32 --keep-csr 0 --device-blocks -1 \
  --steps 1 --warmup 1 --no-cpu-baseline --no-ttk > gpurun_out/r03_bench_c5.json 2> gpurun_out/r03_bench_c5.err; rc=$?
echo "bench c5 rc=$rc"; tail -c 2500 gpurun_out/r03_bench_c5.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 700 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/r03_c5prof -o run -- \
  python bench.py --n 50000000 --basis-bits 32 --keep-csr 0 --device-blocks -1 \
  --steps 1 --warmup 1 --no-cpu-baseline --no-ttk > gpurun_out/r03_c5prof.log 2>&1; rc=$?
echo "prof rc=$rc"; find gpurun_out/r03_c5prof -name "*stats.csv" | head
exit $rc
