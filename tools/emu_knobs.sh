#!/bin/bash
# Emulated G-way shard (1 GPU) under runtime knobs, interleaved: the slowest rank per
# variant.  gpurun -- 'bash tools/emu_knobs.sh <tag> "2 4" c2'
set -o pipefail
T=${1:?tag}; GS=${2:-"2 4"}; C=${3:-c2}
O=gpurun_out/emuk_$T; mkdir -p $O
for r in 1 2; do for g in $GS; do
  for v in "default:" "stage:ZR_BIN_STAGE=1" "serial:ZR_SETUP_OVERLAP=0" "nt256:ZR_TILE_NT=256" "part:"; do
    name=${v%%:*}; envs=${v#*:}; extra=""; [ $name = part ] && extra="--setup partitioned"
    env $envs timeout -k 10 200 python bench.py --config $C --emulate-shard $g $extra --no-cpu-baseline --cold-copies 0 \
      > $O/${name}_${g}_$r.json 2>> $O/err.log || { echo "FAIL $name $g"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/${name}_${g}_$r.json').read().strip().splitlines()[-1]); w=d['ranks'][d['max_rank']]
print('$name G=$g r$r', 't1', d['t1_ms'], 'max', d['max_rank_ms'], 'x', d['speedup'], w['kernels_us'])" | tee -a $O/summary.txt
  done
done; done
