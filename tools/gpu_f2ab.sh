#!/bin/bash
# fused2 A/B of two builds (tools/f2b0, tools/f2b1: F2_DW_PK=0 / 1), default variants, all shapes
set -o pipefail
OUT=gpurun_out/${1:-f2ab}
mkdir -p $OUT
for b in 0 1 0 1; do
  timeout -k 10 200 ./tools/f2b$b 20 "" 0 > $OUT/f2b${b}_$RANDOM.log 2>&1; rc=$?
  echo "== build $b rc=$rc"; ls -t $OUT/f2b${b}_*.log | head -1 | xargs cat | grep -v "^shape"
  case $rc in 124|134|137|139) exit $rc ;; esac
done
exit 0
