# Setup phase-1 timing probe: stamps of the normal build vs loads-only (variant "probe").
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-probe}; mkdir -p $O
L=zenith_amd/variants/probe/libzenith_raster.so
for c in c2 c4; do
ZR_LIB_PATH=$L ZR_DEBUG=128 ZR_DEBUG_TS=$O/st_${c}_full.txt timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/${c}_full.json 2>> $O/err || exit 1
ZR_LIB_PATH=$L ZR_DEBUG=144 ZR_DEBUG_TS=$O/st_${c}_load.txt timeout -k 10 200 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/${c}_load.json 2>> $O/err || exit 2
done
echo done
