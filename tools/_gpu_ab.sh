set -o pipefail
O=gpurun_out/ab22; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for c in c2 c3 cerberus c1; do timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${c}.json 2>>$O/err || exit 3; done
echo done
