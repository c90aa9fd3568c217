# VALU sensitivity of k_tile: +8 / +16 dependent VALU per lane-raster step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v23
mkdir -p $O
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_base.json 2>> $O/bench.err || exit 1
for v in X8 X16; do ZR_LIB_PATH=$PWD/zenith_amd/variants/$v/libzenith_raster.so timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_$v.json 2>> $O/bench.err || exit 2; done
echo done
