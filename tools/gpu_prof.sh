#!/bin/bash
# rocprofv3 kernel-trace summary of a short default bench, then the PMC traffic passes (one call)
set -o pipefail
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-scaling-point > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 $OUT/trace.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_pmc.sh ${1:-prof}_pmc
