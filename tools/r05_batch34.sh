#!/bin/bash
# round 5, batch 34: kernel trace of the bench's time-to-k runs: is the slow-spectrum Ritz
# combination kernel itself slower in the bench (after the matrix is regenerated in the context)?
set -u
mkdir -p gpurun_out/r05_b34
export TMPDIR=/tmp
RBL_RITZ_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r05_b34/prof -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --rmat-steps 0 --c3-steps 0 > gpurun_out/r05_b34/b.json 2> gpurun_out/r05_b34/b.err || { tail -5 gpurun_out/r05_b34/b.err; exit 1; }
grep rbl_ritz gpurun_out/r05_b34/b.err
python3 - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/r05_b34/prof/**/run_kernel_trace.csv", recursive=True) or glob.glob("gpurun_out/r05_b34/prof/run_kernel_trace.csv")
K = list(csv.DictReader(open(f[0])))
tr = [k for k in K if "k_transpose64<true>" in k["Kernel_Name"]]
for t in tr:
    e = int(t["Start_Timestamp"])
    prev = [k for k in K if int(k["End_Timestamp"]) <= e and int(k["End_Timestamp"]) > e - 200e6]
    prev.sort(key=lambda k: int(k["Start_Timestamp"]))
    for k in prev[-4:]:
        print(k["Kernel_Name"][:50], round((int(k["End_Timestamp"]) - int(k["Start_Timestamp"])) / 1e6, 3), "ms, ends", round((e - int(k["End_Timestamp"])) / 1e6, 3), "ms before the transpose")
    print("--")
PY
