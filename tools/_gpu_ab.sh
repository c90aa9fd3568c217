set -o pipefail
O=gpurun_out/ab8; mkdir -p $O
for r in 1 2 3; do for v in 0 1; do ZR_SETUP_SPLIT=$v timeout -k 10 120 python bench.py --no-cpu-baseline > $O/c2_s${v}_$r.json 2>>$O/err || exit 2; done; done
for r in 1 2; do for v in 0 1; do ZR_SETUP_SPLIT=$v timeout -k 10 120 python bench.py --config c3 --no-cpu-baseline > $O/c3_s${v}_$r.json 2>>$O/err || exit 3; done; done
timeout -k 10 120 python bench.py --emulate-shard 4 --no-cpu-baseline > $O/g4_auto.json 2>>$O/err || exit 4
echo done
