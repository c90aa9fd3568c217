# A/B of k_tile variants (loop form, record prefetch, workgroups per CU)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v12
mkdir -p $O
timeout -k 10 700 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_base.json 2>> $O/bench.err || exit 2
for v in L1 PF6 W6 PF6L1 PF8; do
  ZR_LIB_PATH=$PWD/zenith_amd/variants/$v/libzenith_raster.so timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "c2 or small_soup or large or mixed or depth_modes" > $O/pytest_$v.log 2>&1 || exit 3
  ZR_LIB_PATH=$PWD/zenith_amd/variants/$v/libzenith_raster.so timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_$v.json 2>> $O/bench.err || exit 4
done
echo done
