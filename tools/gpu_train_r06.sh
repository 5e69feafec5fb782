#!/bin/bash
# Round-6 training checks on one GPU box: the GPU training tests (accumulator vs reference gradients,
# DDP, bf16 steps), config-5 bench with / without the in-place gradient accumulator, ATen site attribution.
set -o pipefail
TAG=${1:-tr}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_train.py -m gpu -x -v --timeout 600 --timeout-method thread > $OUT/pytest_train.log 2>&1 &&
timeout -k 10 300 python bench.py --train --steps 4 --warmup 1 > $OUT/bench_acc.log 2>&1 &&
TURTLE_TRAIN_ACC=0 timeout -k 10 300 python bench.py --train --steps 4 --warmup 1 > $OUT/bench_noacc.log 2>&1 &&
timeout -k 10 300 python tools/train_sites.py > $OUT/sites.txt 2>&1
rc=$?; tail -3 $OUT/pytest_train.log; grep -h '"value"' $OUT/bench_*.log | cut -c1-200; head -30 $OUT/sites.txt; exit $rc
