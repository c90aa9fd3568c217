# tile-kernel cost breakdown via debug switches (ZR_DEBUG bits: 1 skip raster, 2 skip shade, 8 no LDS atomics, 16 load only)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v10
mkdir -p $O
timeout -k 10 300 python -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "resubmit or c2 or triangle" > $O/pytest.log 2>&1 || exit 1
for d in 0 1 2 8 16; do
  ZR_DEBUG=$d timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_d$d.json 2>> $O/bench.err || exit 2
done
ZR_DEBUG=128 ZR_DEBUG_TS=$O/stamps.txt timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> $O/bench.err || exit 3
echo done
