#!/bin/bash
# 256x256 graph-replay A/B at B = 1 and B = 8 over option sets (';'-separated lists of NAME=VALUE):
#   OPTSETS="gemm9_min_px=0;gemm9_min_px=16384" bash tools/gpu_small_ab.sh <tag>
set -o pipefail
TAG=${1:-small_ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
IFS=';' read -ra SETS <<< "${OPTSETS:-gemm9=1}"
i=0
for set in "${SETS[@]}"; do
  args=""; for o in $set; do args="$args --opt $o"; done
  for b in 1 8; do
    timeout -k 10 300 python -u bench.py --res 256 --batch $b --graph --steps 30 --warmup 5 --no-cpu-baseline --no-psnr --no-scaling-point $args > $OUT/bench_${i}_b$b.log 2>&1
    rc=$?; echo "[$set] B=$b $(tail -1 $OUT/bench_${i}_b$b.log | cut -c1-120)"; [ $rc -ne 0 ] && exit $rc
  done
  i=$((i+1))
done
exit 0
