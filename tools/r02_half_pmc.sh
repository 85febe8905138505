# FETCH_SIZE / WRITE_SIZE of the band-tile SpMM with whole vs half tiles (fuse 3), one pass each.
set -u
mkdir -p gpurun_out/hpmc
export TMPDIR=/tmp
B="python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-ttk --fuse 3"
for h in 0 1; do
  RBL_BT_HALF=$h timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/hpmc/f$h -o b -- $B > gpurun_out/hpmc/f$h.log 2>&1 || exit $?
  RBL_BT_HALF=$h timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d gpurun_out/hpmc/h$h -o b -- $B > gpurun_out/hpmc/h$h.log 2>&1 || exit $?
done
