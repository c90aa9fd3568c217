# hipGraph replay of command lists: parity + bench (graph on/off)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v9
mkdir -p $O
timeout -k 10 700 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_graph.json 2>> $O/bench.err || exit 2
ZR_GRAPH=0 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_nograph.json 2>> $O/bench.err || exit 3
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/kt.log 2>&1 || exit 4
echo done
