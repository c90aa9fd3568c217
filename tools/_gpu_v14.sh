# SQ counters for k_tile: default (nested loop) vs L0 variant
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/v14
mkdir -p $O
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline"
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
Bc="SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_BRANCH SQ_ACTIVE_INST_SCA"
Cc="SQ_THREAD_CYCLES_VALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_LDS_ADDR_CONFLICT SQ_INSTS_LDS_ATOMIC SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"
for v in base L0; do
  if [ $v = L0 ]; then export ZR_LIB_PATH=$PWD/zenith_amd/variants/L0/libzenith_raster.so; fi
  i=0
  for set in "$A" "$Bc" "$Cc"; do
    i=$((i+1))
    timeout -k 10 200 rocprofv3 --pmc $set -d $O/${v}_$i -o run --output-format csv -- $B > $O/${v}_$i.log 2>&1 || exit $i
  done
done
echo done
