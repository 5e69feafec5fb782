#!/bin/bash
# SQ counter passes over tools/f32bench (fp32 GEMM kernels), one rocprofv3 --pmc run per group.
#   bash tools/f32_pmc.sh <tag>   -> gpurun_out/<tag>/p{1,2,3}; report: python3 tools/sq_report.py gpurun_out/<tag> gemm
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-f32pmc}; K="gemm_f32_kernel|gemm_kernelIf"
mkdir -p $OUT
B="./tools/f32bench 2"
timeout -s KILL 90 rocprofv3 --kernel-include-regex "$K" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-include-regex "$K" --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC -f csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-include-regex "$K" --pmc SQ_ACTIVE_INST_MFMA SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_VMEM SQ_INSTS_VMEM -f csv -d $OUT/p3 -o run -- $B > $OUT/p3.log 2>&1
rc=$?; echo "f32_pmc rc=$rc"; python3 tools/sq_report.py $OUT gemm > $OUT/sq_report.txt; exit $rc
