# dynamic-claim setup: parity, then bench per claim batch, then phase stamps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v5
mkdir -p $O
timeout -k 10 700 python -m pytest tests -m gpu -x -q > $O/pytest.log 2>&1 || exit 1
for b in 1 2 4; do
  ZR_SETUP_BATCH=$b timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_b$b.json 2>> $O/bench.err || exit 2
done
ZR_DEBUG=128 ZR_DEBUG_TS=$O/stamps.txt timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_ts.json 2>> $O/bench.err || exit 3
echo done
