#!/bin/bash
# pn GEMM ablations (tools/kbench dbg bits: 1 no stores, 2 no W refills, 4 no LDS reads)
set -o pipefail
OUT=gpurun_out/${1:-kb}
mkdir -p $OUT
for d in 0 1 2 4 3 7; do
  timeout -k 10 120 ./tools/kbench 10 $d > $OUT/kb_$d.log 2>&1; rc=$?
  echo "dbg=$d rc=$rc"; grep -E "L3 GFFW project_in|latent GFFW project_in|L3 qkv" $OUT/kb_$d.log | cut -c1-60
  case $rc in 124|134|137|139) exit $rc ;; esac
done
exit 0
