# HBM traffic per kernel from PMC counters (separate FETCH_SIZE / WRITE_SIZE passes, no
# tracing domains), plus the per-width calibration probe.  Summarise with
#   python tools/pmc_summarize.py gpurun_out/pmc
set -u
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
[ -x tools/pmc_calib_probe ] || /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/pmc_calib.hip -o tools/pmc_calib_probe
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ttk --rmat-steps 0 --c3-steps 0"
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/calib_fetch -o c -- tools/pmc_calib_probe > gpurun_out/pmc/calib_fetch.log 2>&1 \
&& timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/calib_write -o c -- tools/pmc_calib_probe > gpurun_out/pmc/calib_write.log 2>&1 \
&& timeout -k 10 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc/fetch -o b -- $B > gpurun_out/pmc/fetch.log 2>&1 \
&& timeout -k 10 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc/write -o b -- $B > gpurun_out/pmc/write.log 2>&1
rc=$?
echo "pmc rc=$rc"
find gpurun_out/pmc -name "*.csv" | head -20
exit $rc
