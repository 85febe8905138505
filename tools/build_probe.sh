# Build tools/reorth_probe and tools/reorth32_probe against the in-tree librbl_hip.so (its rbl::
# launchers are exported); LD_LIBRARY_PATH=tools/variants/<name> swaps in a variant library.
set -eu
cd "$(dirname "$0")"
for p in reorth_probe reorth32_probe; do
  /opt/rocm/bin/hipcc -O2 -std=c++17 --offload-arch=gfx950 $p.cpp \
    -L../gpu-randomized-block-lanczos_amd/rbl -l:librbl_hip.so \
    -Wl,-rpath,'$ORIGIN/../gpu-randomized-block-lanczos_amd/rbl' -o $p
  echo built tools/$p
done
