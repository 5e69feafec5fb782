#!/bin/bash
# Quick GPU iteration (one gpurun call): parity tests (optionally filtered), the default bench line
# and the per-launch-shape breakdown of its warmup frames. Outputs under gpurun_out/<tag>/.
#   bash tools/gpu_quick.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-q}; K=${2:-}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/$TAG/pytest_gpu.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
TURTLE_BENCH_DUMP=gpurun_out/$TAG/launches.tsv timeout -k 10 400 python -u bench.py --no-cpu-baseline --warmup 3 > gpurun_out/$TAG/bench.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/bench.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
python3 tools/launch_report.py gpurun_out/$TAG/launches.tsv --steps 3 --top 45 > gpurun_out/$TAG/launch_report.txt
head -50 gpurun_out/$TAG/launch_report.txt
