#!/bin/bash
# gffn microbench + SQ counter passes (GPU box): bash tools/gf_pmc.sh <tag>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-gf}
mkdir -p $OUT
timeout -k 10 200 tools/gfbench 20 abl > $OUT/gfbench.log 2>&1; rc=$?; cat $OUT/gfbench.log; [ $rc -ne 0 ] && exit $rc
timeout -s KILL 60 rocprofv3 --kernel-include-regex gffn --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $OUT/p1 -o run -- tools/gfbench 2 prof > $OUT/p1.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --kernel-include-regex gffn --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE -f csv -d $OUT/p2 -o run -- tools/gfbench 2 prof > $OUT/p2.log 2>&1 &&
timeout -s KILL 60 rocprofv3 --kernel-include-regex gffn --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_ACTIVE_INST_MFMA SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_VMEM SQ_INSTS_VMEM -f csv -d $OUT/p3 -o run -- tools/gfbench 2 prof > $OUT/p3.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 tools/sq_report.py $OUT gffn
