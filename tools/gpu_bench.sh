set -u
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --n 1000000 --b 16 --k 20 --steps 2 --no-cpu-baseline > gpurun_out/b1.log 2>&1; rc=$?
echo "bench small rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 900 python bench.py --steps 2 > gpurun_out/b2.log 2>&1; rc=$?
echo "bench full rc=$rc"
exit $rc
