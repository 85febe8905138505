# Alternating same-box A/B of library variants on one bench workload (the reusable form of the
# per-session A/B wrappers of rounds 2-3).
#
# usage: REPS=2 bash tools/ab.sh <tag> "<bench args>" <variant> [<variant> ...]
#   variant = <lib>[:NAME=VAL[:NAME=VAL...]]: <lib> "tree" = the in-tree librbl_hip.so, any other
#   name = tools/variants/<name>/librbl_hip.so (built beforehand with tools/build_variant.sh
#   <name> "<-D defines>"); the NAME=VAL knobs are set for that run (e.g. tree:RBL_BT_HALF=1).
# Each run's bench line goes to gpurun_out/<tag>_<variant>_<rep>.json; one summary line per run
# (value, ms per step, the stage split, the SpMM and partial-reorth rooflines) is printed.
set -u
tag=$1; args=$2; shift 2
REPS=${REPS:-2}
mkdir -p gpurun_out
export TMPDIR=/tmp
for rep in $(seq 1 "$REPS"); do
  for v in "$@"; do
    IFS=':' read -ra parts <<< "$v"
    lib=${parts[0]}
    envs=("${parts[@]:1}")
    unset RBL_LIB
    if [ "$lib" != tree ]; then export RBL_LIB=$PWD/tools/variants/$lib/librbl_hip.so; fi
    safe=$(echo "$v" | tr '=:/' '__-')
    out=gpurun_out/${tag}_${safe}_${rep}.json
    env ${envs[@]+"${envs[@]}"} timeout -k 10 600 python bench.py $args > "$out" 2> "${out%.json}.err" || exit 1
    python - "$v" "$out" <<'PY'
import json, sys
d = json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])
st = {k: round(v, 1) for k, v in d["stage_ms_per_run"].items() if v}
rs = [d["roofline"], d.get("roofline_secondary") or {}]
sp = next((r for r in rs if "spmm" in r.get("kernel", "")), {})
pr = next((r for r in rs if "reorth" in r.get("kernel", "")), {})
print(f"{sys.argv[1]:24s} value={d['value']:.3f} ms/step={d['ms_per_step']:.1f} "
      f"spmm_ms={sp.get('ms_per_launch')} reorth_frac={pr.get('frac')} stages={st}", flush=True)
PY
  done
done
unset RBL_LIB
