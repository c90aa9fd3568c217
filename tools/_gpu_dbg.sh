set -o pipefail
O=gpurun_out/dbg1; mkdir -p $O
ZR_DEBUG=128 ZR_DEBUG_TS=$O/stamps_cerb.txt timeout -k 10 200 python bench.py --config cerberus --steps 3 --warmup 1 --no-cpu-baseline > $O/dbg.json 2>> $O/err || exit 1
echo done
