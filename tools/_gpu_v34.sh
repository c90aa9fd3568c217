# bboxes in LDS, no store drain at the setup barrier
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v34
mkdir -p $O
timeout -k 10 700 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || exit 1
for c in c2 c1 c4; do timeout -k 10 200 python bench.py --config $c --no-cpu-baseline > $O/bench_$c.json 2>> $O/bench.err || exit 2; done
ZR_DEBUG=128 ZR_DEBUG_TS=$O/n.txt timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> $O/bench.err || exit 3
echo done
