#!/bin/bash
# GEMM microbenchmark on the GPU box: tools/kbench (built here) -> gpurun_out/kb.log
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 120 ./tools/kbench ${1:-20} > gpurun_out/kb.log 2>&1
rc=$?; cat gpurun_out/kb.log; exit $rc
