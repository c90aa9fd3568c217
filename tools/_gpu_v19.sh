# per-tile stamps: normal vs reversed tile->block mapping
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v19
mkdir -p $O
ZR_DEBUG=128 ZR_DEBUG_TS=$O/n.txt timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> $O/bench.err || exit 1
ZR_DEBUG=384 ZR_DEBUG_TS=$O/r.txt timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> $O/bench.err || exit 2
ZR_DEBUG=256 timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_r.json 2>> $O/bench.err || exit 3
echo done
