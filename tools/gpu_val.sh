#!/bin/bash
# Validation + measurement on the GPU box (one call): the whole -m gpu suite, smoke(), then the
# default 1080p bench line with its per-launch dump (launch report).
set -o pipefail
OUT=gpurun_out/${1:-val}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 600 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
TURTLE_BENCH_DUMP=$OUT/launches.tsv timeout -k 10 600 python -u bench.py > $OUT/bench_1080p.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench_1080p.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
python3 tools/launch_report.py $OUT/launches.tsv --steps 3 --top 200 > $OUT/launch_report.txt 2>&1
grep "gram\|total" $OUT/launch_report.txt | head -12
exit 0
