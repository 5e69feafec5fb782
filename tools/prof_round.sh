#!/bin/bash
# Profiling recipe run on the GPU box (one gpurun call). Writes under gpurun_out/prof_<tag>/.
#   bash tools/prof_round.sh <tag> [res]
# 1) rocprofv3 --kernel-trace --stats of a short 1080p bench (kernel time summary)
# 2) separate PMC passes (FETCH_SIZE, WRITE_SIZE: one TCC-heavy counter per pass) on the hot
#    kernels; tools/pmc_traffic.py turns them into HBM bytes per launch
set -o pipefail
TAG=${1:-r01}; RES=${2:-1080p}
OUT=gpurun_out/prof_${TAG}
mkdir -p $OUT
export TMPDIR=/tmp
BENCH="bench.py --res $RES --steps 3 --warmup 1 --no-cpu-baseline --no-psnr"
KRE='gemm_pn_kernel|gemm_ar_kernel|gemm_kt_kernel|gemm_lds_kernel|fused2_kernel|fused_kernel|dw_rows_kernel|gram_kernel|sab_'
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 $BENCH > $OUT/trace.log 2>&1 &&
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT/fetch -o run -- python3 $BENCH > $OUT/fetch.log 2>&1 &&
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT/write -o run -- python3 $BENCH > $OUT/write.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
