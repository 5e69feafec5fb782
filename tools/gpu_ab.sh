#!/bin/bash
# One GPU call: optional test run ($TESTS: a pytest -k expression, "all" for the whole -m gpu suite,
# empty to skip), then the 1080p launch breakdown for each option set in $OPTSETS (';'-separated,
# each a space-separated NAME=VALUE list, "-" = defaults), A/B in one process each.
set -o pipefail
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
export TMPDIR=/tmp
if [ -n "$TESTS" ]; then
  K=(); [ "$TESTS" != "all" ] && K=(-k "$TESTS")
  timeout -k 10 1500 python -u -m pytest tests -m gpu -v -x --timeout 600 --timeout-method thread "${K[@]}" > $OUT/pytest_gpu.log 2>&1
  rc=$?; echo "tests rc=$rc"; tail -4 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
IFS=';' read -ra SETS <<< "${OPTSETS:--}"
i=0
for set in "${SETS[@]}"; do
  args=""; [ "$set" != "-" ] && for o in $set; do args="$args --opt $o"; done
  TURTLE_BENCH_DUMP=$OUT/launches_$i.tsv timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-scaling-point ${RESARGS:-} $args > $OUT/bench_$i.log 2>&1
  rc=$?; echo "[$set] $(tail -1 $OUT/bench_$i.log | cut -c1-150)"; [ $rc -ne 0 ] && exit $rc
  python3 tools/launch_report.py $OUT/launches_$i.tsv --steps 3 --top 200 > $OUT/launch_report_$i.txt 2>&1
  i=$((i+1))
done
exit 0
