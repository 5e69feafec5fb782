#!/bin/bash
# PMC passes over tools/kbench (one gpurun call); summaries -> gpurun_out/kpmc/
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/kpmc; mkdir -p $OUT
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
i=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_MFMA SQ_ACTIVE_INST_VALU" \
         "SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES SQ_WAIT_INST_LDS SQ_VMEM_WR_TA_DATA_FIFO_FULL SQ_VMEM_TA_ADDR_FIFO_FULL SQ_INST_LEVEL_VMEM" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -f csv -d $OUT/p$i -o run -- ./tools/kbench 3 > $OUT/p$i.log 2>&1 || echo "pass $i failed"
done
