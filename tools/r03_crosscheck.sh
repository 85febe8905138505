# Round-3 cross-check of the bench line's roofline against rocprofv3: the headline workload
# only (no sub-records, no time-to-k), so every launch of the partial-reorth kernels belongs
# to a timed or warmup 38-step run; per-run kernel time = total / (runs).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03x_prof -o run -- \
  python3 bench.py --steps 3 --warmup 1 --no-ttk --no-cpu-baseline --rmat-steps 0 --c3-steps 0 \
  > gpurun_out/r03x_bench.json 2> gpurun_out/r03x_bench.err; rc=$?
echo "prof rc=$rc"
rm -f gpurun_out/r03x_prof/run_kernel_trace.csv
[ $rc -ne 0 ] && exit $rc
python3 - <<'PY'
import csv, json
rows = list(csv.DictReader(open("gpurun_out/r03x_prof/run_kernel_stats.csv")))
line = json.loads(open("gpurun_out/r03x_bench.json").read().strip().splitlines()[-1])
runs = 4  # 1 warmup + 3 timed, 38 steps each
reo = sum(float(r["TotalDurationNs"]) for r in rows if r["Name"].startswith(("void rbl::k_gram44<32", "void rbl::k_tsmm44f<32")))
spmm = [r for r in rows if r["Name"].startswith("void rbl::k_spmm_bt<32, 9, true, true")]
out = {"bench_part_reorth_ms_per_run": line["roofline"]["ms_per_run"],
       "rocprof_part_reorth_ms_per_run": reo / runs / 1e6,
       "bench_spmm_ms_per_launch": line["roofline_secondary"]["ms_per_launch"],
       "rocprof_spmm_avg_ms": float(spmm[0]["AverageNs"]) / 1e6 if spmm else None,
       "bench_value": line["value"]}
print(json.dumps(out))
open("gpurun_out/r03x_crosscheck.json", "w").write(json.dumps(out, indent=1) + "\n")
PY
