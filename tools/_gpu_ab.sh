set -o pipefail
O=gpurun_out/ab27; mkdir -p $O
for pw in 0 1024 512 256; do for c in c1 cerberus; do
  ZR_SETUP_PER_WG=$pw timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${c}_$pw.json 2>>$O/err || exit 3
done; done
for pw in 0 1024; do ZR_SETUP_PER_WG=$pw timeout -k 10 120 python bench.py --emulate-shard 8 --no-cpu-baseline > $O/g8_$pw.json 2>>$O/err || exit 3; done
echo done
