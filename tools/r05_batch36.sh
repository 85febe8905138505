#!/bin/bash
# round 5, batch 36: is the context's stream still busy when rbl_ritz starts in bench.py's
# slow-spectrum time-to-k?  Trace mode syncs at entry; kernel + memory-copy traces of the run.
set -u
mkdir -p gpurun_out/r05_b36
export TMPDIR=/tmp
RBL_RITZ_TRACE=1 timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d gpurun_out/r05_b36/prof -o run -- \
  python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline --rmat-steps 0 --c3-steps 0 > gpurun_out/r05_b36/b.json 2> gpurun_out/r05_b36/b.err || { tail -5 gpurun_out/r05_b36/b.err; exit 1; }
grep rbl_ritz gpurun_out/r05_b36/b.err
python3 - <<'PY'
import csv, glob
K = list(csv.DictReader(open(glob.glob("gpurun_out/r05_b36/prof/**/run_kernel_trace.csv", recursive=True)[0])))
M = list(csv.DictReader(open(glob.glob("gpurun_out/r05_b36/prof/**/run_memory_copy_trace.csv", recursive=True)[0])))
tr = [k for k in K if "k_transpose64<true>" in k["Kernel_Name"]]
t = tr[-1]; e = int(t["Start_Timestamp"])
ev = [(int(k["Start_Timestamp"]), int(k["End_Timestamp"]), "K " + k["Kernel_Name"][:40]) for k in K] + \
     [(int(m["Start_Timestamp"]), int(m["End_Timestamp"]), "M " + m["Direction"] + " " + str(int(m["End_Timestamp"]) - int(m["Start_Timestamp"]))) for m in M]
ev = [x for x in ev if e - 120e6 <= x[1] <= e + 1e6]
ev.sort()
for s0, e0, name in ev[-25:]:
    print(round((s0 - e) / 1e6, 3), round((e0 - s0) / 1e6, 3), name)
PY
