#!/bin/bash
# fp32 GEMM iteration (one gpurun call): f32bench (new kernel vs gemm_kernel<float>, outputs compared),
# the fp32 GPU tests, and the 540p fp32 bench line (config 3) with its per-launch breakdown.
#   bash tools/gpu_f32.sh <tag> [pytest -k expression]
set -o pipefail
TAG=${1:-f32}; K=${2:-fp32}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 120 ./tools/f32bench 20 > gpurun_out/$TAG/f32bench.log 2>&1
rc=$?; cat gpurun_out/$TAG/f32bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -k "$K" > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
TURTLE_BENCH_DUMP=gpurun_out/$TAG/launches.tsv timeout -k 10 400 python -u bench.py --no-cpu-baseline --res 540p --dtype fp32 --warmup 3 > gpurun_out/$TAG/bench.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/bench.log | cut -c1-400; [ $rc -ne 0 ] && exit $rc
python3 tools/launch_report.py gpurun_out/$TAG/launches.tsv --steps 3 --top 45 > gpurun_out/$TAG/launch_report.txt
head -40 gpurun_out/$TAG/launch_report.txt
