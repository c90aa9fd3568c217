set -o pipefail
O=gpurun_out/ab4; mkdir -p $O
ZR_SETUP_SPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "full_config or small_soup or shards or spill or c4 or determinism or resubmit or mesh" > $O/pytest.log 2>&1 || exit 1
for v in 0 1; do
  for c in c2 c1 c3 c4; do ZR_SETUP_SPLIT=$v timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/s${v}_$c.json 2>>$O/err || exit 2; done
done
echo done
