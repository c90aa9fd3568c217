#!/bin/bash
# Builds libzenith_raster from the sources of git revision <rev> into
# zenith_amd/variants/<name>/ (A/B against an earlier commit with tools/ab.sh).
#   tools/build_rev.sh HEAD~1 prev
set -e
rev=$1; name=$2
root=$(cd "$(dirname "$0")/.." && pwd)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" zenith_amd/csrc include | tar -x -C "$tmp"
out=$root/zenith_amd/variants/$name
mkdir -p "$out"
cd "$tmp/zenith_amd"
F="-O3 -std=c++17 -fPIC -ffp-contract=off -fno-fast-math -fvisibility=hidden -Wall -I../include -Icsrc --offload-arch=gfx950"
/opt/rocm/bin/hipcc $F -x hip -c csrc/zr_runtime.cpp -o "$out/zr_runtime.o"
/opt/rocm/bin/hipcc $F -x hip -c csrc/zr_rccl.cpp -o "$out/zr_rccl.o"
/opt/rocm/bin/hipcc $F -c csrc/zr_kernels.hip -o "$out/zr_kernels.o"
/opt/rocm/bin/hipcc $F -shared -o "$out/libzenith_raster.so" "$out/zr_runtime.o" "$out/zr_rccl.o" "$out/zr_kernels.o" -ldl -Wl,-rpath,/opt/rocm/lib
rm -rf "$tmp"
echo "$out/libzenith_raster.so"
