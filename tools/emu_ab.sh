# A/B of library variants (zenith_amd/variants/<v>) on the 1-GPU emulation of an
# 8-way partitioned tile-row shard (C2, C3): the slowest rank per variant.
#   gpurun -- "VARIANTS=\"a b\" bash tools/emu_ab.sh"
set -o pipefail
O=gpurun_out/emu_ab; mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; echo "pytest rc=$?"; tail -n 2 $O/pytest.log
for r in 1 2; do for c in c2 c3; do for v in ${VARIANTS:-head cur}; do
  ZR_LIB_PATH=zenith_amd/variants/$v/libzenith_raster.so timeout -k 10 200 python bench.py --config $c --emulate-shard 8 --setup partitioned --no-cpu-baseline --cold-copies 0 > $O/${v}_${c}_$r.json 2>> $O/err.log || { echo FAIL $v $c; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/${v}_${c}_$r.json').read().strip().splitlines()[-1]); w=d['ranks'][d['max_rank']]
print('$v $c $r', 't1', d['t1_ms'], 'max', d['max_rank_ms'], 'x', d['speedup'], w['kernels_us'])"
done; done; done
