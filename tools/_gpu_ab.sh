set -o pipefail
O=gpurun_out/ab17; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
K1=$PWD/zenith_amd/variants/k1/libzenith_raster.so
for c in cerberus c1 c2 c3; do
  env ZR_LIB_PATH=$K1 timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${c}_k1.json 2>>$O/err || exit 3
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${c}_k4.json 2>>$O/err || exit 3
done
for g in 4 8; do
  env ZR_LIB_PATH=$K1 timeout -k 10 120 python bench.py --emulate-shard $g --no-cpu-baseline > $O/g${g}_k1.json 2>>$O/err || exit 3
  timeout -k 10 120 python bench.py --emulate-shard $g --no-cpu-baseline > $O/g${g}_k4.json 2>>$O/err || exit 3
done
echo done
