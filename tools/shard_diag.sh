#!/bin/bash
# Emulated 8-way tile-row shards (bench.py --emulate-shard) with the setup chain
# overlapped (production) and serialised (ZR_SETUP_OVERLAP=0: each kernel timed
# alone), for C2 and C3, partitioned and replicated setup.
#   gpurun -- 'bash tools/shard_diag.sh <tag>'
set -o pipefail
T=${1:?tag}; shift
O=gpurun_out/shard_$T
mkdir -p $O
for c in c2 c3; do
  for setup in partitioned replicated; do
    for ov in 1 0; do
      ZR_SETUP_OVERLAP=$ov timeout -k 10 200 python bench.py --config $c --emulate-shard 8 --setup $setup \
        --no-cpu-baseline "$@" > $O/${c}_${setup}_ov$ov.json 2>> $O/err.log || { echo "FAIL $c $setup $ov"; exit 1; }
      echo "$c $setup ov$ov done"
    done
  done
done
python3 - $O <<'PY'
import json, glob, os, sys
for f in sorted(glob.glob(os.path.join(sys.argv[1], "*.json"))):
    d = json.load(open(f))
    print(os.path.basename(f), "T1", d["t1_ms"], "ranks", d["rank_ms"], "speedup", d["speedup"])
    for r in d["ranks"][:2] + d["ranks"][-1:]:
        print("   rank", r["rank"], r["ms"], r["kernels_us"], "pairs", r["bin_pairs"], "setup", r["triangles_setup"])
PY
