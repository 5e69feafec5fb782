#!/bin/bash
# Round-4 GPU check (one gpurun call). Steps are chained: a failing / timed-out step ends the call.
#   bash tools/gpu_r04.sh <tag> [steps...]   steps: tests testsall newtests bench launch prof smoke train trainprof
set -o pipefail
TAG=${1:-r04}; shift
STEPS=${@:-tests bench}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc ;;
    newtests)
      timeout -k 10 600 python -u -m pytest tests/test_dropin_state.py ${KTESTS:-} -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/pytest_new.log 2>&1
      rc=$?; echo "newtests rc=$rc"; tail -3 $OUT/pytest_new.log; [ $rc -ne 0 ] && exit $rc ;;
    ktests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "$KEXPR" > $OUT/pytest_k.log 2>&1
      rc=$?; echo "ktests rc=$rc"; tail -3 $OUT/pytest_k.log; [ $rc -ne 0 ] && exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    bench)
      timeout -k 10 500 python -u bench.py > $OUT/bench_1080p.log 2>&1
      rc=$?; tail -1 $OUT/bench_1080p.log; [ $rc -ne 0 ] && exit $rc ;;
    launch)
      TURTLE_BENCH_DUMP=$OUT/launches.tsv timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-scaling-point $BENCH_EXTRA > $OUT/bench_launch.log 2>&1
      rc=$?; tail -1 $OUT/bench_launch.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
      python3 tools/launch_report.py $OUT/launches.tsv --steps 3 --top 200 > $OUT/launch_report.txt 2>&1; head -30 $OUT/launch_report.txt ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-scaling-point > $OUT/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -1 $OUT/prof.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc ;;
    train)
      timeout -k 10 300 python -u bench.py --train --steps 3 --warmup 1 > $OUT/bench_train.log 2>&1
      rc=$?; tail -1 $OUT/bench_train.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc ;;
    trainprof)
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d $OUT/tprof -o run -- python3 bench.py --train --steps 2 --warmup 1 > $OUT/tprof.log 2>&1
      rc=$?; echo "trainprof rc=$rc"; tail -1 $OUT/tprof.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc ;;
    kbench)
      timeout -k 10 300 $KBENCH_CMD > $OUT/kbench.log 2>&1
      rc=$?; echo "kbench rc=$rc"; tail -30 $OUT/kbench.log; [ $rc -ne 0 ] && exit $rc ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
exit 0
