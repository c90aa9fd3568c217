set -o pipefail
O=gpurun_out/emu4; mkdir -p $O
for g in 2 4 8; do for m in partitioned replicated; do timeout -k 10 120 python bench.py --emulate-shard $g --setup $m --no-cpu-baseline > $O/c2_g${g}_$m.json 2>>$O/err || exit 3; done; done
echo done
