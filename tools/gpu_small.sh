#!/bin/bash
# 256² launch-shape reports (B=1 and B=8, eager, every launch event-timed): one gpurun call.
#   bash tools/gpu_small.sh <tag> [extra bench.py args]
set -o pipefail
TAG=${1:-small}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
for B in 1 8; do
  TURTLE_BENCH_DUMP=$OUT/b$B.tsv timeout -k 10 300 python -u bench.py --res 256 --batch $B --steps 20 --warmup 3 --no-cpu-baseline --no-psnr --no-scaling-point "$@" > $OUT/b$B.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "b$B rc=$rc"; tail -3 $OUT/b$B.log; exit $rc; }
  python3 tools/launch_report.py $OUT/b$B.tsv --steps 3 --top 45 > $OUT/b${B}_report.txt 2>&1
  echo "B=$B: $(tail -1 $OUT/b$B.log | cut -c1-160)"
done
