# Diagnostics: build a copy of librbl_hip.so with extra defines into tools/variants/<name>.so
# usage: bash tools/build_variant.sh <name> "-DRBL_BAND_RD_ABLATE=4"   (run with RBL_LIB=...)
set -eu
name=$1; defs=$2
cd "$(dirname "$0")/../gpu-randomized-block-lanczos_amd/csrc"
mkdir -p ../../tools/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result $defs \
  rbl_api.cpp comm.cpp plan.cpp rowop.hip spmm.hip spmm_window.hip spmm_band.hip tsmm.hip reorth.hip reorth32.hip smallmat.hip gen.hip \
  -x none -shared -L/opt/rocm/lib -lrccl -Wl,-rpath,/opt/rocm/lib -o ../../tools/variants/$name.so
