# PMC HBM traffic (separate FETCH_SIZE / WRITE_SIZE passes, as tools/pmc_traffic.sh) for one
# sub-record workload: bash tools/pmc_traffic_wl.sh <name> <bench args...>
#   rmat:    bash tools/pmc_traffic_wl.sh rmat --matrix rmat
#   circuit: bash tools/pmc_traffic_wl.sh circuit --matrix circuit --n 1585478 --b 16
# Calibration passes are shared with pmc_traffic.sh (gpurun_out/pmc/calib_*).
set -u
name=$1; shift
d=gpurun_out/pmc_$name
mkdir -p $d gpurun_out/pmc
export TMPDIR=/tmp
[ -x tools/pmc_calib_probe ] || /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/pmc_calib_probe
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0 $*"
if [ ! -f gpurun_out/pmc/calib_fetch/c_counter_collection.csv ]; then
  timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/calib_fetch -o c -- tools/pmc_calib_probe > gpurun_out/pmc/calib_fetch.log 2>&1 \
  && timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/calib_write -o c -- tools/pmc_calib_probe > gpurun_out/pmc/calib_write.log 2>&1 || exit 1
fi
cp -r gpurun_out/pmc/calib_fetch gpurun_out/pmc/calib_write $d/
timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $d/fetch -o b -- $B > $d/fetch.log 2>&1 \
&& timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $d/write -o b -- $B > $d/write.log 2>&1
rc=$?
echo "pmc $name rc=$rc"
exit $rc
