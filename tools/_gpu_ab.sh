set -o pipefail
O=gpurun_out/ab24; mkdir -p $O
for c in c3 c1 cerberus c2 c4; do
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${c}_head.json 2>>$O/err || exit 3
  for v in k48 bk b24k; do env ZR_LIB_PATH=$PWD/zenith_amd/variants/$v/libzenith_raster.so timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${c}_$v.json 2>>$O/err || exit 3; done
done
echo done
