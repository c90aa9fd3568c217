#!/bin/bash
# Tile-pass traffic by request class: rocprofv3 FETCH_SIZE passes of
# bench.py with the production library and with the ZR_TILE_DEBUG variant
# (tools/build_variant.sh dbg -DZR_TILE_DEBUG=1, built on the CPU beforehand),
# whose ZR_DEBUG switches each remove one class of the tile pass's reads:
#   2048 identity vertex ids   -> the winners' index gathers
#   4096 every attribute from vertex 0 -> the winners' attribute gathers
#   8192 every resolve record from record 0 -> the resolve's record gathers
#   1    no raster (no list, no record, no winner) -> what is left
# tools/pmc_summary.py --classes turns the differences into bytes per class.
#   gpurun -- 'bash tools/pmc_classes.sh <tag> [bench args...]'
set -o pipefail
export TMPDIR=/tmp
T=${1:?tag}; shift
O=gpurun_out/pmcc_$T
mkdir -p $O
DBG=zenith_amd/variants/dbg/libzenith_raster.so
[ -f $DBG ] || { echo "missing $DBG (tools/build_variant.sh dbg -DZR_TILE_DEBUG=1)"; exit 2; }
run() {  # name lib debug counter
  local n=$1 lib=$2 dbg=$3 ctr=$4
  shift 4
  ZR_LIB_PATH=$lib ZR_DEBUG=$dbg timeout -s KILL 90 rocprofv3 --pmc $ctr -d $O/$n -o run --output-format csv -- \
    python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline --cold-copies 0 --no-census "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc" >> $O/passes.txt
  case $rc in 0) ;; *) echo "pass $n ended with $rc; stopping"; exit $rc;; esac
}
run base_f "" 0 FETCH_SIZE "$@"
run base_w "" 0 WRITE_SIZE "$@"
run dbg0 $DBG 0 FETCH_SIZE "$@"
run ids $DBG 2048 FETCH_SIZE "$@"
run attrs $DBG 4096 FETCH_SIZE "$@"
run recs $DBG 8192 FETCH_SIZE "$@"
run noraster $DBG 1 FETCH_SIZE "$@"
echo done
