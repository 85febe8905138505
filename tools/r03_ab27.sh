# Round-3 A/B 27: fp64 Gram forced to 4 waves per SIMD (tools/variants/g44w4: 128 VGPRs, 15
# spilled) vs 3 (tree: 160 VGPRs).  Reorth probe alternating, 3 reps.
set -u
for rep in 1 2 3; do
  for v in tree g44w4; do
    if [ $v = tree ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=tools/variants/$v; fi
    echo "== $v (rep $rep) $(timeout -k 10 120 ./tools/reorth_probe | tail -1)"
  done
done
