#!/bin/bash
# 256x256 launch breakdown (B = 8 and B = 1, eager) + the graph-replay scaling line
set -o pipefail
OUT=gpurun_out/${1:-small}
mkdir -p $OUT
for b in 8 1; do
  TURTLE_BENCH_DUMP=$OUT/launches_b$b.tsv timeout -k 10 300 python -u bench.py --res 256 --batch $b --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-scaling-point > $OUT/bench_b$b.log 2>&1
  rc=$?; echo "[b=$b] $(tail -1 $OUT/bench_b$b.log | cut -c1-200)"; [ $rc -ne 0 ] && exit $rc
  python3 tools/launch_report.py $OUT/launches_b$b.tsv --steps 3 --top 60 > $OUT/launch_report_b$b.txt 2>&1
done
timeout -k 10 300 python -u bench.py --res 256 --batch 8 --graph --steps 20 --warmup 5 --no-cpu-baseline --no-psnr --no-scaling-point > $OUT/bench_graph_b8.log 2>&1
rc=$?; echo "[graph b=8] $(tail -1 $OUT/bench_graph_b8.log | cut -c1-200)"; exit $rc
