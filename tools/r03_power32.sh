# Round-3: the fp32-basis partial-reorth kernels, basis from HBM vs aliased into cache
# (PROBE_W0=1), times and effective clock (GRBM_GUI_ACTIVE / 8 / wall).
set -u
mkdir -p gpurun_out/r03_power32
export TMPDIR=/tmp
for w0 in 0 1; do
  echo "== PROBE_W0=$w0"
  PROBE_W0=$w0 timeout -k 10 120 ./tools/reorth32_probe | grep -E "nW=36|sum" || exit 1
  PROBE_W0=$w0 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv \
    -d gpurun_out/r03_power32/w$w0 -o c -- ./tools/reorth32_probe > gpurun_out/r03_power32/w$w0.log 2>&1 || { echo "pmc failed"; exit 1; }
  python3 tools/pmc_clock.py gpurun_out/r03_power32/w$w0/c_counter_collection.csv gpurun_out/r03_power32/clock_w$w0.json \
    | grep -A3 '"k_gram32<\|"k_tsmm32f' | grep -E "k_|clock"
done
