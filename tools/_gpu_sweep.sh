# Setup knob sweep (env only, no rebuild): batch and primitives per workgroup on
# C2 and its shard-of-8 emulation.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-sweep}; mkdir -p $O
for kv in "X=0" "ZR_SETUP_BATCH=1" "ZR_SETUP_BATCH=4" "ZR_SETUP_PER_WG=4096" "ZR_SETUP_PER_WG=8192"; do
  n=${kv//=/_}
  env $kv timeout -k 10 120 python bench.py --no-cpu-baseline > $O/c2_$n.json 2>>$O/err || exit 1
  env $kv timeout -k 10 120 python bench.py --no-cpu-baseline --emulate-shard 8 > $O/g8_$n.json 2>>$O/err || exit 2
  env $kv timeout -k 10 120 python bench.py --no-cpu-baseline --config c4 > $O/c4_$n.json 2>>$O/err || exit 3
done
echo done
