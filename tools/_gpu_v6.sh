# setup schedules x batch sizes
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v7
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "c1 or c2 or small_soup or overflow or shards" > $O/pytest.log 2>&1 || exit 1
for sc in 1 2; do for b in 1 2 4; do
  ZR_SETUP_SCHED=$sc ZR_SETUP_BATCH=$b timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_s${sc}_b$b.json 2>> $O/bench.err || exit 2
done; done
ZR_SETUP_SCHED=2 timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "c1 or c2 or small_soup or overflow or shards or c4" > $O/pytest_s2.log 2>&1 || exit 3
for sc in 1 2; do
ZR_SETUP_SCHED=$sc ZR_SETUP_BATCH=2 ZR_DEBUG=128 ZR_DEBUG_TS=$O/stamps_s$sc.txt timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> $O/bench.err || exit 4
done
echo done
