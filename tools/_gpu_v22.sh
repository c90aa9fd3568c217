# 512-thread tiles (8 waves per tile) vs base
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v22
mkdir -p $O
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_base.json 2>> $O/bench.err || exit 1
export ZR_LIB_PATH=$PWD/zenith_amd/variants/T512/libzenith_raster.so
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "c2 or small_soup or large or mixed or depth_modes or c1" > $O/pytest_T512.log 2>&1 || exit 2
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_T512.json 2>> $O/bench.err || exit 3
echo done
