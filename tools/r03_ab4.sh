# Round-3 A/B 4: LDS-DMA staging (tree) vs register staging (tools/variants/gl0): bit identity
# of short runs, PMC groups + FETCH_SIZE / WRITE_SIZE of the partial-reorth kernels (probe),
# two more alternating probe reps.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/bit_tree.npz || exit 1
RBL_LIB=$PWD/tools/variants/gl0/librbl_hip.so timeout -k 10 300 python tools/r03_bitcmp.py dump gpurun_out/bit_gl0.npz || exit 1
python tools/r03_bitcmp.py cmp gpurun_out/bit_tree.npz gpurun_out/bit_gl0.npz
rm -f gpurun_out/bit_*.npz
for v in gl0 tree; do
  if [ $v = tree ]; then unset LD_LIBRARY_PATH; else export LD_LIBRARY_PATH=tools/variants/$v; fi
  bash tools/pmc_groups.sh gpurun_out/r03_pmc_gl_$v ./tools/reorth_probe || exit 1
  i=0
  for g in FETCH_SIZE WRITE_SIZE; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $g --output-format csv -d gpurun_out/r03_pmc_gl_$v/t$i -o p -- \
      ./tools/reorth_probe > gpurun_out/r03_pmc_gl_${v}_t$i.log 2>&1 || { echo "pmc $v $g failed"; exit 1; }
  done
  python tools/pmc_groups_summary.py gpurun_out/r03_pmc_gl_$v k_ > gpurun_out/r03_pmc_gl_$v.txt
done
unset LD_LIBRARY_PATH
rm -rf gpurun_out/r03_pmc_gl_*/g*/*.db
du -sh gpurun_out
