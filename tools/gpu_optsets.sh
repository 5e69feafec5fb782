#!/bin/bash
# 1080p frame A/B on the GPU box (one gpurun call): optional -m gpu tests selected by $KEXPR, then
# the bench line + per-launch report for each option set in $OPTSETS (';'-separated, each a
# space-separated list of NAME=VALUE for turtle_set_option).
#   KEXPR="variants" OPTSETS="gemm9=0;gemm9=1" bash tools/gpu_optsets.sh <tag>
set -o pipefail
TAG=${1:-opts}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$KEXPR" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "$KEXPR" > $OUT/pytest_k.log 2>&1
  rc=$?; echo "ktests rc=$rc"; tail -3 $OUT/pytest_k.log; [ $rc -ne 0 ] && exit $rc
fi
IFS=';' read -ra SETS <<< "${OPTSETS:-gemm9=0}"
i=0
for set in "${SETS[@]}"; do
  args=""; for o in $set; do args="$args --opt $o"; done
  TURTLE_BENCH_DUMP=$OUT/launches_$i.tsv timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-scaling-point $args > $OUT/bench_$i.log 2>&1
  rc=$?; echo "[$set] $(tail -1 $OUT/bench_$i.log | cut -c1-160)"; [ $rc -ne 0 ] && exit $rc
  python3 tools/launch_report.py $OUT/launches_$i.tsv --steps 3 --top 200 > $OUT/launch_report_$i.txt 2>&1
  head -1 $OUT/launch_report_$i.txt
  i=$((i+1))
done
exit 0
