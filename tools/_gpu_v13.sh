# shape-bucket sort + nested row/column lane raster (default) vs incremental loop (L0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v13
mkdir -p $O
timeout -k 10 700 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_base.json 2>> $O/bench.err || exit 2
ZR_LIB_PATH=$PWD/zenith_amd/variants/L0/libzenith_raster.so timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_L0.json 2>> $O/bench.err || exit 3
for c in c1 c4; do timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench.err || exit 4; done
ZR_DEBUG=128 ZR_DEBUG_TS=$O/stamps.txt timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> $O/bench.err || exit 5
echo done
