#!/bin/bash
# PMC passes over tools/dgbench (one counter group per pass), GPU box only:  bash tools/dg_pmc.sh [shape 0|1]
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/dgpmc
mkdir -p $OUT
S=${1:-0}
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $OUT/p1 -o run -- tools/dgbench 3 $S > $OUT/p1.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC -f csv -d $OUT/p2 -o run -- tools/dgbench 3 $S > $OUT/p2.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_MFMA SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_VMEM SQ_INSTS_VMEM -f csv -d $OUT/p3 -o run -- tools/dgbench 3 $S > $OUT/p3.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -f csv -d $OUT/p4 -o run -- tools/dgbench 3 $S > $OUT/p4.log 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -f csv -d $OUT/p5 -o run -- tools/dgbench 3 $S > $OUT/p5.log 2>&1
rc=$?; echo "pmc rc=$rc"; python3 tools/kpmc_report.py $OUT; exit $rc
