set -o pipefail
O=gpurun_out/dr1; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "depth_range or viewport" --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
echo done
