#!/bin/bash
# 1-GPU shard emulation lines (bench.py --emulate-shard): every rank timed beside T1.
#   gpurun -- 'bash tools/emu_shards.sh <tag> [configs] [shard counts]'
set -o pipefail
export TMPDIR=/tmp
T=${1:?tag}; C=${2:-"c2 c3"}; GS=${3:-"8"}
O=gpurun_out/emu_$T
mkdir -p $O
for c in $C; do
  for g in $GS; do
    for s in replicated partitioned; do
      timeout -k 10 240 python bench.py --config $c --emulate-shard $g --setup $s --no-cpu-baseline \
        > $O/${c}_g${g}_$s.json 2>> $O/err.log || { echo "FAIL $c $g $s"; exit 1; }
      python3 -c "import json,sys; d=json.load(open('$O/${c}_g${g}_$s.json')); print('$c G=$g $s', 't1', d['t1_ms'], 'max', d['max_rank_ms'], 'speedup', d['speedup'], 'ranks', d['rank_ms'])"
    done
  done
done
