# PMC traffic of the C4b (R-MAT) and C3-shape workloads, summarised per workload
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/pmc_traffic_wl.sh rmat --matrix rmat || exit 1
python tools/pmc_summarize.py gpurun_out/pmc_rmat gpurun_out/pmc_rmat.json "rmat 10000000 32 38" || exit 1
bash tools/pmc_traffic_wl.sh circuit --matrix circuit --n 1585478 --b 16 --k 20 || exit 1
python tools/pmc_summarize.py gpurun_out/pmc_circuit gpurun_out/pmc_circuit.json "circuit 1585478 16 75" || exit 1
find gpurun_out -name "*.db" -delete
find gpurun_out -name "*kernel_trace*" -delete
du -sh gpurun_out
