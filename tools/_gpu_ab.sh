set -o pipefail
O=gpurun_out/ab10; mkdir -p $O
B="ZR_LIB_PATH=$PWD/zenith_amd/variants/base/libzenith_raster.so"
for r in 1 2; do for c in cerberus c2 c4; do
  env ZR_LIB_PATH=$PWD/zenith_amd/variants/base/libzenith_raster.so timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${c}_base_$r.json 2>>$O/err || exit 3
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${c}_new_$r.json 2>>$O/err || exit 3
done; done
echo done
