# 32-B compact records (+ prefetch variant)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v27
mkdir -p $O
timeout -k 10 700 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || exit 1
for c in c2 c1 c4; do timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench.err || exit 2; done
export ZR_LIB_PATH=$PWD/zenith_amd/variants/PF8/libzenith_raster.so
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "c2 or small_soup or large or mixed or c1" > $O/pytest_PF8.log 2>&1 || exit 3
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_PF8.json 2>> $O/bench.err || exit 4
echo done
