#!/bin/bash
# Training step on one GPU box: rocprofv3 kernel stats of a 3-step config-5 bench and their family summary
# (ATen call sites with forward origins first: tools/train_sites.py).
set -o pipefail
TAG=${1:-tp}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$SITES" ] && timeout -k 10 400 python tools/train_sites.py > $OUT/sites.txt 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --train --steps 3 --warmup 1 > $OUT/bench_prof.log 2>&1
rc=$?
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1)
[ -n "$f" ] && cp "$f" $OUT/train_kernel_stats.csv && python3 tools/train_prof_summary.py $OUT/train_kernel_stats.csv 40 > $OUT/train_prof_summary.txt
rm -rf $OUT/prof                                 # the kernel trace itself is too large to bring back
tail -3 $OUT/bench_prof.log; cat $OUT/train_prof_summary.txt | head -70; exit $rc
