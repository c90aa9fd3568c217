#!/bin/bash
# Emulated 8-way shards under environment variants (runtime knobs), interleaved:
#   gpurun -- 'bash tools/emu_env_ab.sh <tag> "c2 c3" partitioned "ZR_TILE_NT=0" "ZR_TILE_NT=512" ...'
set -o pipefail
T=${1:?tag}; C=${2:?configs}; SETUP=${3:?setup}; shift 3
O=gpurun_out/emu_$T
mkdir -p $O
for c in $C; do
  i=0
  for v in "$@"; do
    i=$((i+1))
    env $(echo "$v" | tr ',' ' ') timeout -k 10 200 python bench.py --config $c --emulate-shard 8 --setup $SETUP \
      --no-cpu-baseline > $O/${c}_v$i.json 2>> $O/err.log || { echo "FAIL $c $v"; exit 1; }
    python3 -c "
import json,sys; d=json.load(open('$O/${c}_v$i.json'))
print('$c', '$v', 'T1', d['t1_ms'], 'max rank', d['max_rank_ms'], 'speedup', d['speedup'], 'spread', round(max(d['rank_ms'])/min(d['rank_ms'])-1,3))
r=d['ranks'][d['max_rank']]; print('   worst rank kernels', r['kernels_us'])"
  done
done
