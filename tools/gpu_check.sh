set -u
mkdir -p gpurun_out
rocminfo 2>/dev/null | grep -m3 -E "gfx|Marketing" > gpurun_out/rocminfo.txt
timeout -k 10 600 python -m pytest tests -m gpu -q --timeout 300 > gpurun_out/t1.log 2>&1; rc=$?
echo "pytest rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --n 1000000 --b 16 --k 20 --steps 2 --no-cpu-baseline > gpurun_out/b1.log 2>&1; rc=$?
echo "bench small rc=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python bench.py --steps 2 > gpurun_out/b2.log 2>&1; rc=$?
echo "bench full rc=$rc"
exit $rc
