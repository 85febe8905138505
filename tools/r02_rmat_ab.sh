# A/B of SpMM variants on the R-MAT workload (C4b): bench.py against tools/variants/<name>
# (RBL_LIB) and the in-tree library, alternating.  Usage: bash tools/r02_rmat_ab.sh v1 [v2 ...]
set -u
mkdir -p gpurun_out
run() {
  timeout -k 10 300 python bench.py --matrix rmat --steps 1 --warmup 1 --no-cpu-baseline --no-ttk \
    > gpurun_out/rmat_ab_$1.json 2> gpurun_out/rmat_ab_$1.err || return $?
  python3 -c "import json;d=json.load(open('gpurun_out/rmat_ab_$1.json'));r=d['roofline_secondary'] if 'spmm' in d['roofline_secondary']['kernel'] else d['roofline'];print('$1', d['value'], 'iters/s', r['ms_per_launch'], 'ms/SpMM')"
}
for rep in 1 2; do
  for v in "$@"; do
    test -f tools/variants/$v/librbl_hip.so || { echo "missing $v"; exit 3; }
    RBL_LIB=tools/variants/$v/librbl_hip.so run ${v}_$rep || exit $?
  done
  run tree_$rep || exit $?
done
