#!/bin/bash
# Profiling recipe run on the GPU box (one gpurun call). Writes under gpurun_out/prof_<tag>/.
#   bash tools/prof_round.sh <tag> [res]
# 1) rocprofv3 --kernel-trace --stats of a short 1080p bench (kernel time summary)
# 2) separate PMC passes (FETCH_SIZE, WRITE_SIZE, SQ stall counters) on the hot kernels only
set -o pipefail
TAG=${1:-r01}; RES=${2:-1080p}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="bench.py --res $RES --steps 3 --warmup 1 --no-cpu-baseline --no-psnr"
KRE='gemm_panel_kernel|gemm_kernel|fused_kernel|dw_kernel|gram_kernel|sab_'
timeout -k 10 300 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT/fetch -o run -- python3 $BENCH > $OUT/fetch.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT/write -o run -- python3 $BENCH > $OUT/write.log 2>&1 &&
timeout -k 10 400 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS --kernel-include-regex "$KRE" -f csv -d $OUT/sq -o run -- python3 $BENCH > $OUT/sq.log 2>&1
