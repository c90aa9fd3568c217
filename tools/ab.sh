#!/bin/bash
# A/B timing of library variants (tools/build_variant.sh) on the GPU box:
#   gpurun -- 'bash tools/ab.sh <tag> "base zp" "c2 c1" 2 [extra bench args]'
# Variants run interleaved per repetition; every bench run has its own time limit
# and the first failure ends the script.  Summary: gpurun_out/ab_<tag>/summary.txt
set -o pipefail
T=${1:?tag}; V=${2:?variants}; C=${3:?configs}; R=${4:-2}; shift 4
O=gpurun_out/ab_$T
mkdir -p $O
for r in $(seq $R); do
  for c in $C; do
    for v in $V; do
      # a variant is a build name, optionally with environment settings: name:VAR=1,VAR2=2
      lib=zenith_amd/variants/${v%%:*}/libzenith_raster.so
      [ "${v%%:*}" = prod ] && lib=zenith_amd/lib/libzenith_raster.so  # the in-tree build
      envs=""; [ "$v" != "${v#*:}" ] && envs=$(echo "${v#*:}" | tr ',' ' ')
      env $envs ZR_LIB_PATH=$lib timeout -k 10 150 python bench.py --config $c --no-cpu-baseline --cold-copies 0 "$@" \
        > "$O/$(echo $v | tr ":=," "---")_${c}_$r.json" 2>> $O/err.log || { echo "FAIL $v $c $r"; exit 1; }
      echo "$v $c $r done"
    done
  done
done
python tools/ab_summary.py $O | tee $O/summary.txt
