set -o pipefail
O=gpurun_out/ab3; mkdir -p $O
for n in 0 32 48 64 96; do
  ZR_SETUP_CUS=$n timeout -k 10 120 python bench.py --no-cpu-baseline > $O/c2_cus$n.json 2>>$O/err || exit 2
done
ZR_SETUP_CUS=64 timeout -k 10 120 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "full_config or resubmit or small_soup" > $O/pytest.log 2>&1 || exit 3
for c in c1 c3 c4; do timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${c}.json 2>>$O/err || exit 4; done
ZR_DEBUG=128 ZR_DEBUG_TS=$O/stamps_c2.txt timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/dbg.json 2>> $O/err || exit 6
echo done
