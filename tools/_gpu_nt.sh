# k_tile workgroup size A/B (environment only): ZR_TILE_NT=256 / 512 on C1-C3.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-nt}; mkdir -p $O
for nt in 256 512; do for c in c1 c2 c3; do
  ZR_TILE_NT=$nt timeout -k 10 120 python bench.py --no-cpu-baseline --config $c > $O/${c}_$nt.json 2>>$O/err || exit 1
done; done
echo done
