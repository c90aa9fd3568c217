#!/bin/bash
# Tile-edge A/B on the GPU box (round 6): GPU parity of the in-tree
# build and of the 16- and 64-px variants (tools/build_variant.sh t16 -DZR_TILE=16,
# t64 -DZR_TILE=64), then interleaved bench lines and the emulated 8-way shards.
#   gpurun --timeout 1800 -- 'bash tools/tile_ab.sh [variants]'
# A test failure of a variant is recorded (its log) and the A/B goes on; a crash
# (not exit 0/1) ends the script.
set -o pipefail
V=${1:-t16 t64}
O=gpurun_out/tile_ab; mkdir -p $O
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_prod.log 2>&1 || { echo "prod pytest failed"; exit 1; }
tail -n 1 $O/pytest_prod.log
for v in $V; do
  ZR_LIB_PATH=zenith_amd/variants/$v/libzenith_raster.so timeout -k 10 400 python -u -m pytest tests -m gpu -q --maxfail=8 \
    --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1
  rc=$?; echo "$v pytest rc=$rc: $(tail -n 1 $O/pytest_$v.log)"
  [ $rc -le 1 ] || exit 2
done
bash tools/ab.sh tile "prod $V" "c2 c1 c4 cerberus c2x c3" 2 || exit 3
for r in 1 2; do for c in c2 c3; do for s in partitioned replicated; do for v in prod $V; do
  lib=zenith_amd/variants/$v/libzenith_raster.so; [ $v = prod ] && lib=zenith_amd/lib/libzenith_raster.so
  ZR_LIB_PATH=$lib timeout -k 10 200 python bench.py --config $c --emulate-shard 8 --setup $s --no-cpu-baseline --cold-copies 0 \
    > $O/emu_${v}_${c}_${s}_$r.json 2>> $O/emu_err.log || { echo "FAIL emu $v $c $s"; exit 4; }
  python3 -c "
import json; d=json.loads(open('$O/emu_${v}_${c}_${s}_$r.json').read().strip().splitlines()[-1]); w=d['ranks'][d['max_rank']]
print('$v $c $s $r', 't1', d['t1_ms'], 'max', d['max_rank_ms'], 'x', d['speedup'], w['kernels_us'])" | tee -a $O/emu_summary.txt
done; done; done; done
echo done
