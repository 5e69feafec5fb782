#!/bin/bash
# HIP-graph serving mode: parity vs eager, then 256^2 / 1080p bench lines with and without graphs.
set -o pipefail
mkdir -p gpurun_out/graph
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_hip_configs.py -m gpu -x -v --timeout 200 --timeout-method thread -k graphed > gpurun_out/graph/t.log 2>&1
rc=$?; tail -4 gpurun_out/graph/t.log; [ $rc -ne 0 ] && exit $rc
for a in "--res 256" "--res 256 --graph" "--res 256 --batch 8 --graph" "--graph"; do
  timeout -k 10 300 python -u bench.py $a --no-cpu-baseline --no-psnr > gpurun_out/graph/b.log 2>&1 || exit $?
  echo "$a"; tail -1 gpurun_out/graph/b.log | cut -c1-330; tail -1 gpurun_out/graph/b.log >> gpurun_out/graph/lines.jsonl
done
