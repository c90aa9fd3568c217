# k_tile workgroup size A/B, repeated: C2 and C4 at ZR_TILE_NT=256 / 512.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${1:-nt2}; mkdir -p $O
for r in 1 2; do for nt in 256 512; do for c in c2 c4; do
  ZR_TILE_NT=$nt timeout -k 10 120 python bench.py --no-cpu-baseline --config $c > $O/${c}_${nt}_$r.json 2>>$O/err || exit 1
done; done; done
echo done
