set -o pipefail
O=gpurun_out/ab5; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_all.log 2>&1 || exit 1
for v in base nowide; do
  L=""; [ $v != base ] && L=zenith_amd/variants/$v/libzenith_raster.so
  for c in c2 c1 c3 cerberus; do ZR_LIB_PATH=$L timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${v}_$c.json 2>>$O/err || exit 2; done
done
echo done
