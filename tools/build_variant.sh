#!/bin/bash
# Builds an A/B variant of libzenith_raster with extra -D knobs into
# zenith_amd/variants/<name>/ (load it with ZR_LIB_PATH=... for tests / bench.py).
#   tools/build_variant.sh dbg -DZR_TILE_DEBUG=1
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/zenith_amd/variants/$name
mkdir -p "$out"
cd "$root/zenith_amd"
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fvisibility=hidden -Wall -I../include -Icsrc --offload-arch=gfx950 $*"
/opt/rocm/bin/hipcc $F -x hip -c csrc/zr_runtime.cpp -o "$out/zr_runtime.o"
/opt/rocm/bin/hipcc $F -x hip -c csrc/zr_rccl.cpp -o "$out/zr_rccl.o"
/opt/rocm/bin/hipcc $F -c csrc/zr_kernels.hip -o "$out/zr_kernels.o" -Rpass-analysis=kernel-resource-usage 2> "$out/resource-usage.txt"
/opt/rocm/bin/hipcc $F -shared -o "$out/libzenith_raster.so" "$out/zr_runtime.o" "$out/zr_rccl.o" "$out/zr_kernels.o" -ldl -Wl,-rpath,/opt/rocm/lib
echo "$out/libzenith_raster.so"
