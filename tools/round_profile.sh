# Round-end evidence for the default bench line: the bench JSON, the rocprofv3 kernel-trace
# summary of the SAME command, the PMC traffic passes (FETCH_SIZE / WRITE_SIZE) and the
# effective-clock pass (GRBM_GUI_ACTIVE).  Usage: bash tools/round_profile.sh <tag>
set -u
tag=${1:-latest}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err || exit $?
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$tag -o run --output-format csv -- python3 bench.py > gpurun_out/prof_$tag.log 2>&1 || exit $?
bash tools/pmc_traffic.sh || exit $?
timeout -s KILL 300 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc_clk -o c -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ttk > gpurun_out/pmc_clk.log 2>&1 || exit $?
echo done
