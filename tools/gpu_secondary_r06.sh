#!/bin/bash
# Round-6 secondary bench lines (one gpurun call): 256^2 B = 8 and B = 1 graph replay (config 2 / the
# scaling workload), TurtleSuper 4x SR (config 4), 540p fp32 (config 3), training (config 5).
set -o pipefail
TAG=${1:-r06s}
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() { local name=$1; shift; timeout -k 10 400 python -u bench.py --no-cpu-baseline "$@" > $OUT/$name.log 2>&1; local rc=$?;
        echo "$name rc=$rc"; grep '"value"' $OUT/$name.log | cut -c1-200; return $rc; }
run train --train --steps 6 --warmup 2 &&
run b8 --res 256 --batch 8 --graph --no-psnr --no-scaling-point &&
run b1 --res 256 --graph --no-psnr --no-scaling-point &&
run sr --sr --no-psnr --no-scaling-point &&
run fp32_540p --res 540p --dtype fp32 --no-psnr --no-scaling-point
rc=$?
cat $OUT/*.log | grep '"value"' > $OUT/secondary.jsonl; exit $rc
