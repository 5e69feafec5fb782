#!/bin/bash
# 256x256 B=8 graph-replay A/B (the --gpus N scaling workload) over option sets (';'-separated, each a
# space-separated list of NAME=VALUE for turtle_set_option):
#   OPTSETS="attn_fin=0;attn_fin=1" bash tools/gpu_optsets_small.sh <tag>
set -o pipefail
TAG=${1:-small_opts}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
IFS=';' read -ra SETS <<< "${OPTSETS:-gemm9=1}"
i=0
for set in "${SETS[@]}"; do
  args=""; for o in $set; do args="$args --opt $o"; done
  timeout -k 10 300 python -u bench.py --res 256 --batch 8 --graph --steps 30 --warmup 5 --no-cpu-baseline --no-psnr --no-scaling-point $args > $OUT/bench_$i.log 2>&1
  rc=$?; echo "[$set] $(tail -1 $OUT/bench_$i.log | cut -c1-140)"; [ $rc -ne 0 ] && exit $rc
  i=$((i+1))
done
exit 0
