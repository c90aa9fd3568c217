# attribute k_tile VALU work by debug skips (1 skip raster, 2 skip shade, 16 load only)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v15
mkdir -p $O
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline"
for d in 0 1 2 16; do
  ZR_DEBUG=$d timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_BRANCH -d $O/d$d -o run --output-format csv -- $B > $O/d$d.log 2>&1 || exit 1
done
echo done
