set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r06c
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06c/pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/r06c/pytest.log; [ $rc -le 1 ] || exit 1
bash tools/ab.sh front2 "prod nofront r05" "c2x c3x c2 c3 c1 cerberus c4" 2 || exit 2
ZR_LIB_PATH=zenith_amd/variants/r04/libzenith_raster.so bash tools/pmc_probe.sh r04c3 --config c3 > /dev/null || exit 3
ZR_LIB_PATH=zenith_amd/variants/r05/libzenith_raster.so bash tools/pmc_probe.sh r05c3 --config c3 > /dev/null || exit 4
ZR_TILE=32 bash tools/pmc_probe.sh r06c3 --config c3 > /dev/null || exit 5
echo done
