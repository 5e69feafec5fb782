#!/bin/bash
# training-kernel launch-size sweep (tools/train_kbench.py under TURTLE_TRAIN_TUNE settings)
set -o pipefail
TAG=${1:-kbs}
OUT=gpurun_out/$TAG
mkdir -p $OUT
for t in 0,0,0 256,128,1024 1024,512,512 384,64,4096; do
  TURTLE_TRAIN_TUNE=$t timeout -k 10 120 python tools/train_kbench.py > $OUT/tune_$t.txt 2>&1 || exit $?
done
TURTLE_TRAIN_ABL=1 timeout -k 10 120 python tools/train_kbench.py > $OUT/abl.txt 2>&1
for f in $OUT/tune_*.txt $OUT/abl.txt; do echo "== $f"; grep -E "ln_bwd\+res|colsum|dw_wgrad" $f; done
