#!/bin/bash
# tilepd microbench + SQ counter passes (GPU box): bash tools/tp_pmc.sh <tag> [shape]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-tp}; S=${2:-0}
mkdir -p $OUT
timeout -k 10 120 tools/tpbench 20 > $OUT/tpbench.log 2>&1; rc=$?; cat $OUT/tpbench.log; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 60 rocprofv3 --kernel-include-regex tilepd --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $OUT/p1 -o run -- tools/tpbench 2 $S > $OUT/p1.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --kernel-include-regex tilepd --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC -f csv -d $OUT/p2 -o run -- tools/tpbench 2 $S > $OUT/p2.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --kernel-include-regex tilepd --pmc SQ_ACTIVE_INST_MFMA SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_VMEM SQ_INSTS_VMEM -f csv -d $OUT/p3 -o run -- tools/tpbench 2 $S > $OUT/p3.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
