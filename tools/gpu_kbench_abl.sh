#!/bin/bash
# pn GEMM ablations / stamps: tools/kbench with debug bits (1 no stores, 2 no W refills, 4 no LDS reads, 8 stamps)
set -o pipefail
mkdir -p gpurun_out
for d in ${@:-0 8}; do
  echo "== dbg $d" >> gpurun_out/kba.log
  timeout -k 10 120 ./tools/kbench 10 $d >> gpurun_out/kba.log 2>&1 || exit $?
done
