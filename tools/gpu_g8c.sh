#!/bin/bash
# gemm8 ablation table only (GPU box)
set -o pipefail
OUT=gpurun_out/${1:-g8c}
mkdir -p $OUT
timeout -k 10 240 ./tools/g8abl 10 abl > $OUT/g8abl.log 2>&1; rc=$?; cat $OUT/g8abl.log; exit $rc
