set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-perf}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_all.log 2>&1 || exit 1
for c in c2 c1 cerberus; do timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/$c.json 2>>$O/err || exit 2; done
timeout -k 10 120 python bench.py --emulate-shard 8 --no-cpu-baseline > $O/c2_g8.json 2>>$O/err || exit 3
ZR_DEBUG=128 ZR_DEBUG_TS=$O/stamps_c2.txt timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/dbg.json 2>> $O/err || exit 6
echo done
