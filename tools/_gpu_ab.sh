set -o pipefail
O=gpurun_out/ab14; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for r in 1 2; do
  env ZR_LIB_PATH=$PWD/zenith_amd/variants/q/libzenith_raster.so timeout -k 10 120 python bench.py --emulate-shard 4 --no-cpu-baseline > $O/g4_q_$r.json 2>>$O/err || exit 3
  timeout -k 10 120 python bench.py --emulate-shard 4 --no-cpu-baseline > $O/g4_head_$r.json 2>>$O/err || exit 3
  timeout -k 10 120 python bench.py --emulate-shard 8 --no-cpu-baseline > $O/g8_head_$r.json 2>>$O/err || exit 3
  timeout -k 10 120 python bench.py --no-cpu-baseline > $O/c2_head_$r.json 2>>$O/err || exit 3
done
echo done
