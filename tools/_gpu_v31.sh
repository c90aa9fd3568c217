# rotated phase-2 atomics; setup + tile stamps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v31
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "c2 or overflow or shards or small_soup" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench.json 2>> $O/bench.err || exit 2
ZR_DEBUG=128 ZR_DEBUG_TS=$O/n.txt timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> $O/bench.err || exit 3
echo done
