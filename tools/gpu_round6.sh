#!/bin/bash
# Round-6 evidence on the current sources (one gpurun call): smoke(), the default bench line (CPU
# baseline + the 1080p oracle pin), the rocprofv3 kernel-trace stats and the PMC traffic passes.
#   bash tools/gpu_round6.sh <tag>
set -o pipefail
TAG=${1:-r06}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py > $OUT/bench_1080p.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench_1080p.log | cut -c1-600; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_evidence.sh ${TAG}_ev
