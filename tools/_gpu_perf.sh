set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-perf}; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_all.log 2>&1 || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline > $O/c2.json 2>>$O/err || exit 2
timeout -k 10 120 python bench.py --config c1 --no-cpu-baseline > $O/c1.json 2>>$O/err || exit 2
for g in 2 8; do timeout -k 10 120 python bench.py --emulate-shard $g --no-cpu-baseline > $O/c2_g${g}.json 2>>$O/err || exit 3; done
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt8 -o run --output-format csv -- python3 bench.py --emulate-shard 8 --steps 50 --warmup 5 --no-cpu-baseline > $O/kt8.log 2>&1 || exit 4
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt1 -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/kt1.log 2>&1 || exit 5
ZR_DEBUG=128 ZR_DEBUG_TS=$O/stamps8.txt timeout -k 10 200 python bench.py --emulate-shard 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/dbg.json 2>> $O/err || exit 6
echo done
