set -o pipefail
O=gpurun_out/ab26; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
H=$PWD/zenith_amd/variants/head/libzenith_raster.so
for r in 1 2; do for c in c2 c1 c3 cerberus; do
  env ZR_LIB_PATH=$H timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${c}_head_$r.json 2>>$O/err || exit 3
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${c}_new_$r.json 2>>$O/err || exit 3
done; done
echo done
