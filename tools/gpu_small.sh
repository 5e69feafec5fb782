#!/bin/bash
# Small-frame runs (one gpurun call): 256^2 B=1 / B=8, eager and graph, plus the per-launch
# breakdown of the B=1 eager warmup frames. Outputs under gpurun_out/<tag>/.
set -o pipefail
TAG=${1:-small}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
for cfg in "--batch 1" "--batch 1 --graph" "--batch 8 --graph"; do
  timeout -k 10 300 python -u bench.py --res 256 $cfg --steps 50 --warmup 5 --no-cpu-baseline --no-psnr >> gpurun_out/$TAG/bench256.log 2>&1 || exit $?
  tail -1 gpurun_out/$TAG/bench256.log | cut -c1-160
done
TURTLE_BENCH_DUMP=gpurun_out/$TAG/launches.tsv timeout -k 10 300 python -u bench.py --res 256 --steps 5 --warmup 3 --no-cpu-baseline --no-psnr > gpurun_out/$TAG/dump.log 2>&1 || exit $?
python3 tools/launch_report.py gpurun_out/$TAG/launches.tsv --steps 3 --top 40 > gpurun_out/$TAG/launch_report.txt
head -30 gpurun_out/$TAG/launch_report.txt
