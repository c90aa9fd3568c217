set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/prof1; mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 bench.py --emulate-shard 8 --steps 50 --warmup 5 --no-cpu-baseline > $O/kt.log 2>&1 || exit 1
ZR_DEBUG=128 ZR_DEBUG_TS=$O/stamps.txt timeout -k 10 200 python bench.py --emulate-shard 8 --steps 3 --warmup 1 --no-cpu-baseline > $O/dbg.json 2>> $O/err || exit 2
ZR_DEBUG=128 ZR_DEBUG_TS=$O/stamps_rep.txt timeout -k 10 200 python bench.py --emulate-shard 8 --setup replicated --steps 3 --warmup 1 --no-cpu-baseline > $O/dbg_rep.json 2>> $O/err || exit 3
echo done
