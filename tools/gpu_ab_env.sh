#!/bin/bash
# A/B of one environment switch on the 1080p bench (one gpurun call): default, then with the
# given VAR=VALUE, each with the per-launch breakdown. Outputs under gpurun_out/<tag>/.
#   bash tools/gpu_ab_env.sh <tag> VAR=VALUE
set -o pipefail
TAG=${1:-ab}; KV=${2:?VAR=VALUE}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
TURTLE_BENCH_DUMP=gpurun_out/$TAG/a.tsv timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-psnr --warmup 3 > gpurun_out/$TAG/a.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/a.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
env "$KV" TURTLE_BENCH_DUMP=gpurun_out/$TAG/b.tsv timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-psnr --warmup 3 > gpurun_out/$TAG/b.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/b.log | cut -c1-200; [ $rc -ne 0 ] && exit $rc
python3 tools/launch_report.py gpurun_out/$TAG/a.tsv --steps 3 --top 60 > gpurun_out/$TAG/a_report.txt
python3 tools/launch_report.py gpurun_out/$TAG/b.tsv --steps 3 --top 60 > gpurun_out/$TAG/b_report.txt
head -1 gpurun_out/$TAG/a_report.txt; head -1 gpurun_out/$TAG/b_report.txt
