#!/bin/bash
# 1080p default-switch re-check on the final sources (one box): the default line, then one switch
# changed at a time, default again at the end (drift check)
set -o pipefail
TAG=${1:-osw}
OUT=gpurun_out/$TAG
mkdir -p $OUT
B="bench.py --no-cpu-baseline --no-psnr --no-scaling-point --no-roofline"
i=0
for o in "" "gffn_c128=0" "tilepd=0" "gemm9=2" "gemm9=0" "sab_waves=4" "sab_waves=8" "dwgemm=0" "gemm8=0" "gemm_kt=0" "ffn=0" ""; do
  i=$((i+1))
  args=""; [ -n "$o" ] && args="--opt $o"
  timeout -k 10 200 python $B $args > $OUT/run_$i.log 2>&1 || { echo "run $i ($o) failed"; exit 1; }
  echo "${o:-default}: $(grep -o '"value": [0-9.]*' $OUT/run_$i.log)"
done
