set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v26
mkdir -p $O
ZR_DEBUG=128 ZR_DEBUG_TS=$O/n.txt timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> $O/bench.err || exit 1
echo done
