#!/bin/bash
# Round-4 kernel bring-up on the GPU box (one gpurun call): gemm8 microbenchmark + race screen, the
# SAB score block-size sweep, the switch-variant parity tests, then the 1080p launch breakdown for
# each option set in $OPTSETS (';'-separated, each a space-separated list of NAME=VALUE).
#   OPTSETS="gemm8=0;gemm8=1" bash tools/gpu_g8.sh <tag>
set -o pipefail
TAG=${1:-g8}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 ./tools/g8bench 20 > $OUT/g8bench.log 2>&1
rc=$?; cat $OUT/g8bench.log; [ $rc -ne 0 ] && exit $rc
for w in 4 8; do
  timeout -k 10 120 ./tools/sabbench 10 0 $w > $OUT/sabbench_w$w.log 2>&1
  rc=$?; grep "dbg=0" $OUT/sabbench_w$w.log; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 120 ./tools/sabbench 10 8 4 > $OUT/sabbench_s8.log 2>&1
rc=$?; grep "dbg=0" $OUT/sabbench_s8.log; [ $rc -ne 0 ] && exit $rc
if [ -z "$NOTESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "${KEXPR:-variants}" > $OUT/pytest_k.log 2>&1
  rc=$?; echo "ktests rc=$rc"; tail -3 $OUT/pytest_k.log; [ $rc -ne 0 ] && exit $rc
fi
IFS=';' read -ra SETS <<< "${OPTSETS:-gemm8=0;gemm8=1;gemm8=2}"
i=0
for set in "${SETS[@]}"; do
  args=""; for o in $set; do args="$args --opt $o"; done
  TURTLE_BENCH_DUMP=$OUT/launches_$i.tsv timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-scaling-point $args > $OUT/bench_$i.log 2>&1
  rc=$?; echo "[$set] $(tail -1 $OUT/bench_$i.log | cut -c1-160)"; [ $rc -ne 0 ] && exit $rc
  python3 tools/launch_report.py $OUT/launches_$i.tsv --steps 3 --top 200 > $OUT/launch_report_$i.txt 2>&1
  i=$((i+1))
done
exit 0
