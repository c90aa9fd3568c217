# PMC A/B: HEAD (64-B records) vs compact records
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v29
mkdir -p $O
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline"
for v in cur HEAD; do
  if [ $v = HEAD ]; then export ZR_LIB_PATH=$PWD/zenith_amd/variants/HEAD/libzenith_raster.so; fi
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_ANY SQ_INSTS_VMEM_WR -d $O/${v}_1 -o run --output-format csv -- $B > $O/${v}_1.log 2>&1 || exit 1
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE -d $O/${v}_2 -o run --output-format csv -- $B > $O/${v}_2.log 2>&1 || exit 2
  timeout -k 10 200 rocprofv3 --pmc TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum -d $O/${v}_3 -o run --output-format csv -- $B > $O/${v}_3.log 2>&1 || exit 3
done
echo done
