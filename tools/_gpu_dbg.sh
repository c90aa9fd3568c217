set -o pipefail
O=gpurun_out/dbg2; mkdir -p $O
for v in 0 16 1 2 3; do ZR_DEBUG=$v timeout -k 10 120 python bench.py --no-cpu-baseline > $O/d$v.json 2>>$O/err || exit 1; done
echo done
