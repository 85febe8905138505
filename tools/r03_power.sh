# Round-3 power experiment: the partial-reorth kernels with the basis streamed from HBM (probe
# default) vs every panel aliasing panel 0 (PROBE_W0=1: same instructions, basis from L2 /
# Infinity Cache), times and the effective clock (GRBM_GUI_ACTIVE / 8 / wall).
set -u
mkdir -p gpurun_out/r03_power
export TMPDIR=/tmp
for rep in 1 2; do
  for w0 in 0 1; do
    echo "== PROBE_W0=$w0 (rep $rep)"
    PROBE_W0=$w0 timeout -k 10 120 ./tools/reorth_probe | grep -E "nW=36|sum" || exit 1
  done
done
for w0 in 0 1; do
  PROBE_W0=$w0 timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv \
    -d gpurun_out/r03_power/w$w0 -o c -- ./tools/reorth_probe > gpurun_out/r03_power/w$w0.log 2>&1 || { echo "pmc w0=$w0 failed"; exit 1; }
  python3 tools/pmc_clock.py gpurun_out/r03_power/w$w0/c_counter_collection.csv gpurun_out/r03_power/clock_w$w0.json \
    | grep -A3 '"k_gram44\|"k_tsmm44f' | grep -E "k_|clock|avg" 
done
