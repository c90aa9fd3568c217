set -o pipefail
O=gpurun_out/emu3; mkdir -p $O
timeout -k 10 120 python bench.py --no-cpu-baseline > $O/c2.json 2>>$O/err || exit 1
timeout -k 10 120 python bench.py --no-cpu-baseline --force-dist > $O/c2_dist1.json 2>>$O/err || exit 2
for g in 2 4 8; do for m in partitioned replicated; do timeout -k 10 120 python bench.py --emulate-shard $g --setup $m --no-cpu-baseline > $O/c2_g${g}_$m.json 2>>$O/err || exit 3; done; done
for g in 8; do timeout -k 10 120 python bench.py --config c3 --emulate-shard $g --no-cpu-baseline > $O/c3_g${g}.json 2>>$O/err || exit 4; done
echo done
