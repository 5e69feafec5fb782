#!/bin/bash
# Instruction-mix / stall PMC passes for the kernels matching a regex (one gpurun call).
#   bash tools/prof_kernel.sh '<kernel regex>' <tag> [res]
set -o pipefail
KRE=$1; TAG=${2:-k}; RES=${3:-1080p}
OUT=gpurun_out/pk_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="bench.py --res $RES --steps 1 --warmup 0 --no-cpu-baseline --no-psnr"
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES"
P2="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR"
P3="SQ_WAVES SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_INST_LEVEL_VMEM SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-include-regex "$KRE" -f csv -d $OUT/p$i -o run -- python3 $BENCH > $OUT/p$i.log 2>&1 || exit $?
done
