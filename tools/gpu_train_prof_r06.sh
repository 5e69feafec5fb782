#!/bin/bash
# Training step attribution on one GPU box: ATen sites with forward origins (anomaly mode), then the
# rocprofv3 kernel stats of a 3-step config-5 bench and their family summary.
set -o pipefail
TAG=${1:-tp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python tools/train_sites.py > $OUT/sites.txt 2>&1 &&
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 bench.py --train --steps 3 --warmup 1 > $OUT/bench_prof.log 2>&1
rc=$?
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" $OUT/train_kernel_stats.csv && python3 tools/train_prof_summary.py $OUT/train_kernel_stats.csv 40 > $OUT/train_prof_summary.txt
head -45 $OUT/sites.txt; cat $OUT/train_prof_summary.txt | head -60; exit $rc
