set -o pipefail
O=gpurun_out/ab25; mkdir -p $O
for b in 2 4 1; do ZR_SETUP_BATCH=$b timeout -k 10 120 python bench.py --config c4 --no-cpu-baseline > $O/c4_b$b.json 2>>$O/err || exit 3; done
for b in 2 4; do ZR_SETUP_BATCH=$b timeout -k 10 120 python bench.py --config c2 --no-cpu-baseline > $O/c2_b$b.json 2>>$O/err || exit 3; done
ZR_DEBUG=128 ZR_DEBUG_TS=$O/st.txt timeout -k 10 200 python bench.py --config c4 --steps 2 --warmup 1 --no-cpu-baseline > $O/d.json 2>> $O/err || exit 2
echo done
