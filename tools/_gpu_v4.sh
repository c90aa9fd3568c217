# round-1 v4: parity (incl. C example + gloo shards on GPU) + bench + kernel-trace stats
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v4
mkdir -p $O
timeout -k 10 700 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || exit 1
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || exit 2
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --steps 50 --warmup 5 --no-cpu-baseline > $O/kt.log 2>&1 || exit 3
echo done
