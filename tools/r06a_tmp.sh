set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06d/pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/r06d/pytest.log; [ $rc -le 1 ] || exit 1
for c in c3 cerberus; do
ZR_LIB_PATH=zenith_amd/variants/r04/libzenith_raster.so bash tools/pmc_probe.sh r04_$c --config $c > /dev/null || exit 3
ZR_LIB_PATH=zenith_amd/variants/r05/libzenith_raster.so bash tools/pmc_probe.sh r05_$c --config $c > /dev/null || exit 4
ZR_TILE=32 bash tools/pmc_probe.sh r06_$c --config $c > /dev/null || exit 5
done
echo done
