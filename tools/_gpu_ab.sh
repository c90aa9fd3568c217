set -o pipefail
O=gpurun_out/rot1; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || exit 1
for r in 1 2; do for c in c2 cerberus c1; do timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > $O/${c}_$r.json 2>>$O/err || exit 3; done; done
ZR_TILE_NT=512 timeout -k 10 120 python bench.py --config cerberus --no-cpu-baseline > $O/cerb512.json 2>>$O/err || exit 3
echo done
