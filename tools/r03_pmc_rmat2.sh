# PMC traffic of the C4b (R-MAT) workload after the seg-kernel occupancy change
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_rmat
bash tools/pmc_traffic_wl.sh rmat --matrix rmat || exit 1
python tools/pmc_summarize.py gpurun_out/pmc_rmat gpurun_out/pmc_rmat.json "rmat 10000000 32 38" || exit 1
find gpurun_out -name "*.db" -delete
