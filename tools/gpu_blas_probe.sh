#!/bin/bash
# One gpurun call: GEMM + depthwise microbenchmarks, then the 1080p bench with and without hipBLASLt
# (per-launch breakdowns under gpurun_out/<tag>/).
set -o pipefail
TAG=${1:-bp}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 120 ./tools/kbench 20 > gpurun_out/$TAG/kb.log 2>&1 && cat gpurun_out/$TAG/kb.log &&
timeout -k 10 120 ./tools/dwbench 20 > gpurun_out/$TAG/dw.log 2>&1 && cat gpurun_out/$TAG/dw.log || exit $?
for v in blas noblas; do
  if [ $v = noblas ]; then export TURTLE_NO_BLASLT=1; fi
  TURTLE_BENCH_DUMP=gpurun_out/$TAG/launches_$v.tsv timeout -k 10 400 python -u bench.py --no-cpu-baseline --warmup 3 > gpurun_out/$TAG/bench_$v.log 2>&1
  rc=$?; tail -1 gpurun_out/$TAG/bench_$v.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
  python3 tools/launch_report.py gpurun_out/$TAG/launches_$v.tsv --steps 3 --top 60 > gpurun_out/$TAG/launch_report_$v.txt
done
exit 0
