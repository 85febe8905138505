# Round-3 A/B 12: Gram splits 3..6 x CUs by rows (tree, >= 4096 rows per split) vs 3 x CUs
# (tools/variants/splits1), probe at n = 1e7, 4e6, 1.25e6.
set -u
mkdir -p gpurun_out
for n in 10000000 4000000 1250000; do
  for rep in 1 2; do
    for v in splits1 tree; do
      echo "== n=$n $v (rep $rep)"
      if [ $v = tree ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=tools/variants/$v; fi
      timeout -k 10 120 ./tools/reorth_probe $n > gpurun_out/r03_ab12_${n}_${v}_$rep.log || exit 1
      grep -E "nW=36|sum" gpurun_out/r03_ab12_${n}_${v}_$rep.log
    done
  done
done
