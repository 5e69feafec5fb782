#!/bin/bash
# fused-kernel microbenchmark with ablation bits: bash tools/gpu_fbench.sh "0 1 2 4 8 15"
set -o pipefail
mkdir -p gpurun_out
for d in ${1:-0}; do
  echo "== dbg $d" >> gpurun_out/fb.log
  timeout -k 10 120 ./tools/fbench 10 $d >> gpurun_out/fb.log 2>&1 || exit $?
done
