#!/bin/bash
# One GPU round trip: parity tests, then the 1080p bench with a per-launch dump (gpurun_out/).
#   bash tools/gpu_check.sh [pytest -k expr]
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
K=${1:-}
if [ -n "$K" ]; then KARG=(-k "$K"); else KARG=(); fi
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread "${KARG[@]}" > gpurun_out/t.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/t.log
[ $rc -ne 0 ] && exit $rc
rm -f gpurun_out/launches.tsv
TURTLE_BENCH_DUMP=gpurun_out/launches.tsv timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/b.log 2>&1
rc=$?; tail -1 gpurun_out/b.log; [ $rc -ne 0 ] && exit $rc
# (optional) kernel-trace summary of a short run: GPU_CHECK_PROF=1
if [ -n "$GPU_CHECK_PROF" ]; then
  rm -rf gpurun_out/prof
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-psnr > gpurun_out/p.log 2>&1
  echo "prof rc=$?"
fi
