#!/bin/bash
# SQ / TCC counter passes over bench.py on the GPU box (one pass per counter set,
# each under its own time limit).  A pass that fails with an ordinary error (an
# unknown counter name) is skipped; a pass that times out, aborts or faults ends
# the script.
#   gpurun -- 'bash tools/pmc_probe.sh <tag> [bench args...]'   (PMC_SET=mem: the memory-pipeline set)
# Output: gpurun_out/pmc_<tag>/<pass>/run_counter_collection.csv, summarised by
# tools/pmc_table.py into gpurun_out/pmc_<tag>/summary.txt.
set -o pipefail
export TMPDIR=/tmp
T=${1:?tag}; shift
O=gpurun_out/pmc_$T
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1
if [ "${PMC_SET:-sq}" = mem ]; then
PASSES=(
  "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE GRBM_COUNT"
  "TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum"
  "TD_BUSY_avr TD_TC_STALL_sum"
  "TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_LATENCY_sum"
  "TCC_EA0_RDREQ_LEVEL_sum TCC_EA0_RDREQ_sum TCC_HIT_sum TCC_MISS_sum"
  "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_READ_sum TCP_UTCL1_TRANSLATION_MISS_sum"
  "SQ_INSTS_VMEM_RD SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES"
)
else
PASSES=(
  "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA"
  "SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_LDS_IDX_ACTIVE SQ_INSTS_SMEM SQ_ACTIVE_INST_FLAT SQ_INSTS_BRANCH"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
  "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"
  "TA_BUSY_avr TA_TA_BUSY_sum GRBM_GUI_ACTIVE GRBM_COUNT"
)
fi
i=0
for p in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $p -d $O/p$i -o run --output-format csv -- python3 bench.py --steps 20 --warmup 10 --no-cpu-baseline --cold-copies 0 --no-census "$@" > $O/p$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc: $p" >> $O/passes.txt
  case $rc in 124|137|134|139) echo "pass $i ended with $rc; stopping"; exit $rc;; esac
done
python3 tools/pmc_table.py $O > $O/summary.txt 2>&1
cat $O/summary.txt
