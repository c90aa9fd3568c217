set -o pipefail
O=gpurun_out/part2; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -v --timeout 300 --timeout-method thread -k "partitioned or spill" > $O/pytest.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --force-dist > $O/c2_dist1.json 2>>$O/err || exit 2
for g in 2 4 8; do timeout -k 10 120 python bench.py --emulate-shard $g --no-cpu-baseline > $O/c2_g${g}.json 2>>$O/err || exit 3; done
timeout -k 10 120 python bench.py --config c3 --emulate-shard 8 --no-cpu-baseline > $O/c3_g8.json 2>>$O/err || exit 4
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_all.log 2>&1 || exit 5
echo done
