set -o pipefail
mkdir -p gpurun_out/r06b
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r06b/pytest.log 2>&1; rc=$?; tail -n 3 gpurun_out/r06b/pytest.log; [ $rc -le 1 ] || exit 1
bash tools/ab.sh front "prod nohiz nofront r05" "c2x c3x c3 c4 c1 c2 cerberus" 2 || exit 2
bash tools/ab.sh regr "prod:ZR_TILE=32 r04 r05" "c1 c3 cerberus" 2 || exit 3
