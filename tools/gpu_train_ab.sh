#!/bin/bash
# same-box A/B of a training-step env switch: bench.py --train alternately without / with it, twice each
set -o pipefail
TAG=${1:-tab}; VAR=${2:-TURTLE_NG_SLIM}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for i in 1 2; do
  for v in 0 1; do
    env $VAR=$v timeout -k 10 300 python bench.py --train --steps 6 --warmup 2 > $OUT/b_${v}_$i.log 2>&1 || exit $?
    echo "$VAR=$v run $i: $(grep -o '"value": [0-9.]*' $OUT/b_${v}_$i.log)"
  done
done
