#!/bin/bash
# Secondary bench lines of the BASELINE configs (one gpurun call) -> gpurun_out/<tag>/secondary.jsonl
set -o pipefail
TAG=${1:-sec}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
run() {
  timeout -k 10 $1 python -u bench.py "${@:2}" > $OUT/line.log 2>&1 || { echo "failed: ${*:2}"; tail -5 $OUT/line.log; exit 1; }
  tail -1 $OUT/line.log >> $OUT/secondary.jsonl; tail -1 $OUT/line.log | cut -c1-200
}
run 300 --res 256 --graph --steps 50 --warmup 5 --no-cpu-baseline
run 300 --res 256 --batch 8 --graph --steps 20 --warmup 3 --no-cpu-baseline
run 400 --sr --no-cpu-baseline
run 400 --res 540p --dtype fp32 --no-cpu-baseline --no-psnr
run 500 --train --steps 3 --warmup 1
