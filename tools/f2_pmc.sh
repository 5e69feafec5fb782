#!/bin/bash
# PMC passes over tools/f2bench (one counter group per pass), GPU box only:
#   bash tools/f2_pmc.sh <shape-substring> <variant>
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/f2pmc
mkdir -p $OUT
S=${1:-"L1 GFFW"}; V=${2:-1}
timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $OUT/p1 -o run -- tools/f2bench 3 "$S" $V > $OUT/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC -f csv -d $OUT/p2 -o run -- tools/f2bench 3 "$S" $V > $OUT/p2.log 2>&1
rc=$?; echo "pmc rc=$rc"; exit $rc
