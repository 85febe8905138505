# Diagnostics: build a copy of librbl_hip.so with extra defines into
# tools/variants/<name>/librbl_hip.so (run against it with LD_LIBRARY_PATH=tools/variants/<name>,
# or RBL_LIB=tools/variants/<name>/librbl_hip.so for the Python package).
# usage: bash tools/build_variant.sh <name> "-DRBL_G44_ROWS=32"
set -eu
name=$1; defs=$2
cd "$(dirname "$0")/../gpu-randomized-block-lanczos_amd/csrc"
out=../../tools/variants/$name
mkdir -p $out/obj
srcs=$(sed -n 's/^SRCS := //p' Makefile)
pids=""
for s in $srcs; do
  o=$out/obj/${s%.*}.o
  if [ "${s##*.}" = "cpp" ]; then x="-x hip"; else x=""; fi
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-result -Wno-unused-value $defs $x -c $s -o $o &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
/opt/rocm/bin/hipcc -fPIC --offload-arch=gfx950 $out/obj/*.o -shared -L/opt/rocm/lib \
  -lrocprofiler-sdk-roctx -Wl,-rpath,/opt/rocm/lib -o $out/librbl_hip.so
rm -rf $out/obj
echo "built $out/librbl_hip.so"
