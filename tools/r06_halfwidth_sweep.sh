#!/bin/bash
# round 6: the SpMM beyond the 64-band. n = 1e7, ~100 nonzeros per row
# (1 + p 2H: p = 99 / 2H), b = 32, one GPU: per half-width the kernel the library picks, its ms
# per launch and frac on SURVEY's CSR bytes (bench.py's SpMM roofline), C4a runs only.
# Usage: tools/r06_halfwidth_sweep.sh <outdir> [half-widths...] [-- extra bench args]
set -u
out=${1:-gpurun_out/r06_hw}; shift || true
hws=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do hws+=("$1"); shift; done
[ "${1:-}" = "--" ] && shift
[ ${#hws[@]} -eq 0 ] && hws=(64 128 256 512 1024 2048)
mkdir -p $out
export TMPDIR=/tmp
for H in "${hws[@]}"; do
  p=$(python3 -c "print(round(99 / (2 * $H), 6))")
  timeout -k 10 300 python bench.py --halfwidth $H --density $p --steps 2 --warmup 1 \
    --rmat-steps 0 --c3-steps 0 --no-cpu-baseline --no-ttk "$@" > $out/hw$H.json 2> $out/hw$H.err; rc=$?
  [ $rc -ne 0 ] && { echo "H=$H rc=$rc"; tail -20 $out/hw$H.err; exit $rc; }
  python3 - $out/hw$H.json $H <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = next(x for x in (d["roofline"], d["roofline_secondary"]) if x["kernel"].startswith("spmm"))
print(f"H={sys.argv[2]:>5} nnz={d['config']['nnz']} kernel={r['kernel']} fmt={r['matrix_format']} "
      f"ms/launch={r['ms_per_launch']} frac={r['frac']} value={d['value']} "
      f"gathers_gbs={r.get('gbs_incl_q_row_gathers')}", flush=True)
PY
done
