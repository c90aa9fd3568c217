# overlapped draws (setup stream + two scratch sets)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v30
mkdir -p $O
timeout -k 10 700 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || exit 1
for c in c2 c1 c4; do timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench.err || exit 2; done
ZR_OVERLAP=0 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_nooverlap.json 2>> $O/bench.err || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/kt.log 2>&1 || exit 4
echo done
