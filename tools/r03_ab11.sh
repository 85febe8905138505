# Round-3 A/B 11: twice the Gram splits (tools/variants/splits2, 6 x CUs) vs the tree (3 x CUs),
# probe at n = 1e7 and n = 1.25e6.
set -u
mkdir -p gpurun_out
for n in 10000000 1250000; do
  for rep in 1 2; do
    for v in splits2 tree; do
      echo "== n=$n $v (rep $rep)"
      if [ $v = tree ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=tools/variants/$v; fi
      timeout -k 10 120 ./tools/reorth_probe $n > gpurun_out/r03_ab11_${n}_${v}_$rep.log || exit 1
      grep -E "nW= 2 |nW=18|nW=36|sum" gpurun_out/r03_ab11_${n}_${v}_$rep.log
    done
  done
done
