# A/B of the partial-reorth kernels: the probe against tools/variants/<name>/librbl_hip.so
# (LD_LIBRARY_PATH takes precedence over the probe's RUNPATH) and the in-tree library,
# alternating, on the same box.  Usage: bash tools/r02_reorth_ab.sh name1 [name2 ...]
set -u
mkdir -p gpurun_out
for rep in ${REPS:-1 2}; do
  for v in "$@"; do
    echo "== $v (rep $rep)"
    test -f tools/variants/$v/librbl_hip.so || { echo "missing variant $v"; exit 3; }
    LD_LIBRARY_PATH=tools/variants/$v timeout -k 10 120 ./tools/reorth_probe | tail -2 || exit $?
  done
  echo "== tree (rep $rep)"
  timeout -k 10 120 ./tools/reorth_probe | tail -2 || exit $?
done
