set -o pipefail
O=gpurun_out/ab1; mkdir -p $O
for v in base nolpt; do
  L=""; [ $v != base ] && L=zenith_amd/variants/$v/libzenith_raster.so
  for c in c1 c2 c3; do ZR_LIB_PATH=$L timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${v}_$c.json 2>>$O/err || exit 1; done
  ZR_LIB_PATH=$L timeout -k 10 120 python bench.py --emulate-shard 8 --no-cpu-baseline > $O/${v}_c2g8.json 2>>$O/err || exit 2
done
echo done
