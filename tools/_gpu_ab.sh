set -o pipefail
O=gpurun_out/ab16; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for r in 1 2; do timeout -k 10 120 python bench.py --config cerberus --no-cpu-baseline > $O/cerb_$r.json 2>>$O/err || exit 3; done
echo done
