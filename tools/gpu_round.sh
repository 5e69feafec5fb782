#!/bin/bash
# Round-end style GPU check (one gpurun call): parity tests, the default bench line (with the CPU
# baseline and PSNR), then a rocprofv3 kernel-trace summary of a short bench. Outputs: gpurun_out/.
#   bash tools/gpu_round.sh <tag>
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > gpurun_out/$TAG/pytest_gpu.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/$TAG/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/$TAG/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/$TAG/bench_1080p.log 2>&1
rc=$?; tail -1 gpurun_out/$TAG/bench_1080p.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d gpurun_out/$TAG/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr > gpurun_out/$TAG/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/$TAG/prof.log; exit $rc
