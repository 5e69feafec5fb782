#!/bin/bash
# Round-3 GPU check (one gpurun call). Steps are chained: a failing / timed-out step ends the call.
#   bash tools/gpu_r03.sh <tag> [tests|train|bench|prof ...]
set -o pipefail
TAG=${1:-r03}; shift
STEPS=${@:-tests train bench}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
      rc=$?; echo "tests rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc ;;
    testsall)
      # every GPU test, no -x (one pass shows every failure); $DESELECT: extra --deselect ids
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread $DESELECT > $OUT/pytest_gpu.log 2>&1
      rc=$?; echo "testsall rc=$rc"; tail -3 $OUT/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc ;;
    vprobe)
      timeout -k 10 300 python -u tools/variant_probe.py > $OUT/vprobe.log 2>&1
      rc=$?; echo "vprobe rc=$rc"; cat $OUT/vprobe.log | grep dB; [ $rc -ne 0 ] && exit $rc ;;
    quick)
      timeout -k 10 600 python -u -m pytest tests -m gpu -v -x --timeout 300 --timeout-method thread -k "dropin or train" > $OUT/pytest_quick.log 2>&1
      rc=$?; echo "quick rc=$rc"; tail -3 $OUT/pytest_quick.log; [ $rc -ne 0 ] && exit $rc ;;
    parity)
      timeout -k 10 600 python -u -m pytest tests/test_hip_parity.py -v -x --timeout 300 --timeout-method thread -k "variants or biasfree or bf16_psnr or gopro" > $OUT/pytest_parity.log 2>&1
      rc=$?; echo "parity rc=$rc"; tail -3 $OUT/pytest_parity.log; [ $rc -ne 0 ] && exit $rc ;;
    smoke)
      timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
      rc=$?; echo "smoke rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    train)
      timeout -k 10 300 python -u bench.py --train --steps 3 --warmup 1 > $OUT/bench_train.log 2>&1
      rc=$?; tail -1 $OUT/bench_train.log; [ $rc -ne 0 ] && exit $rc
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/trainprof -o run -- python3 bench.py --train --steps 2 --warmup 1 > $OUT/trainprof.log 2>&1
      rc=$?; echo "trainprof rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    bench)
      timeout -k 10 500 python -u bench.py > $OUT/bench_1080p.log 2>&1
      rc=$?; tail -1 $OUT/bench_1080p.log; [ $rc -ne 0 ] && exit $rc ;;
    prof)
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -f csv -d $OUT/prof -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-scaling-point > $OUT/prof.log 2>&1
      rc=$?; echo "prof rc=$rc"; tail -1 $OUT/prof.log; [ $rc -ne 0 ] && exit $rc ;;
    launch)
      TURTLE_BENCH_DUMP=$OUT/launches.tsv timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-scaling-point > $OUT/bench_launch.log 2>&1
      rc=$?; tail -1 $OUT/bench_launch.log; [ $rc -ne 0 ] && exit $rc
      python3 tools/launch_report.py $OUT/launches.tsv --steps 3 > $OUT/launch_report.txt 2>&1 ;;
    modprobe)
      timeout -k 10 500 python -u tools/psnr_probe.py --seeds 3 --subsets --by-module --frames 2 > $OUT/psnr_modules.log 2>&1
      rc=$?; echo "modprobe rc=$rc"; [ $rc -ne 0 ] && exit $rc ;;
    ab)
      # launch-shape reports of the default build and kernel-switch variants (AB_OPTS, ';'-separated)
      IFS=';' read -ra VARS <<< "${AB_OPTS:-;gemm9=0}"
      i=0
      for v in "${VARS[@]}"; do
        extra=""; for o in $v; do extra="$extra --opt $o"; done
        TURTLE_BENCH_DUMP=$OUT/ab$i.tsv timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-scaling-point $extra > $OUT/ab$i.log 2>&1
        rc=$?; [ $rc -ne 0 ] && { echo "ab $i rc=$rc"; tail -3 $OUT/ab$i.log; exit $rc; }
        python3 tools/launch_report.py $OUT/ab$i.tsv --steps 3 > $OUT/ab${i}_report.txt 2>&1
        echo "ab $i [$v]: $(python3 -c "import json,sys; d=json.loads(open('$OUT/ab$i.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'])")"
        i=$((i+1))
      done ;;
    pmcpdw)
      K=${PMC_KERNEL:-fused2_kernel}
      B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --no-scaling-point --no-roofline"
      timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $OUT/pmc/p1 -o run -- $B > $OUT/pmc_p1.log 2>&1 &&
      timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC -f csv -d $OUT/pmc/p2 -o run -- $B > $OUT/pmc_p2.log 2>&1 &&
      timeout -s KILL 120 rocprofv3 --kernel-include-regex $K --pmc SQ_ACTIVE_INST_MFMA SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_VMEM SQ_INSTS_VMEM -f csv -d $OUT/pmc/p3 -o run -- $B > $OUT/pmc_p3.log 2>&1
      rc=$?; echo "pmc rc=$rc"; python3 tools/kpmc_report.py $OUT/pmc > $OUT/pmc_report.txt 2>&1; head -20 $OUT/pmc_report.txt; [ $rc -ne 0 ] && exit $rc ;;
    f2b)
      timeout -k 10 300 ./tools/f2bench ${F2B_REPS:-20} "${F2B_ONLY:-}" ${F2B_V:-0} > $OUT/f2bench.log 2>&1
      rc=$?; echo "f2b rc=$rc"; cat $OUT/f2bench.log; [ $rc -ne 0 ] && exit $rc ;;
    f2old)
      timeout -k 10 300 ./tools/f2bench_old ${F2B_REPS:-20} "${F2B_ONLY:-}" ${F2B_V:-0} > $OUT/f2bench_old.log 2>&1
      rc=$?; echo "f2old rc=$rc"; cat $OUT/f2bench_old.log; [ $rc -ne 0 ] && exit $rc ;;
    tprof)
      timeout -k 10 400 python -u tools/train_prof.py > $OUT/train_prof.txt 2>&1
      rc=$?; echo "tprof rc=$rc"; tail -40 $OUT/train_prof.txt | head -5; [ $rc -ne 0 ] && exit $rc ;;
    tcopy)
      timeout -k 10 300 python -u tools/train_copies.py --gpu --res 128 --batch 2 --frames 2 > $OUT/train_copies.txt 2>&1
      rc=$?; echo "tcopy rc=$rc"; head -30 $OUT/train_copies.txt; [ $rc -ne 0 ] && exit $rc ;;
    pmc)
      timeout -k 10 900 bash tools/gpu_pmc.sh $TAG/pmc > $OUT/pmc.log 2>&1
      rc=$?; echo "pmc rc=$rc"; tail -3 $OUT/pmc.log; [ $rc -ne 0 ] && exit $rc ;;
    iso)
      timeout -k 10 300 python -u tools/bf16_isolate.py > $OUT/iso.log 2>&1
      rc=$?; echo "iso rc=$rc"; cat $OUT/iso.log | grep PSNR; [ $rc -ne 0 ] && exit $rc ;;
    tdebug)
      HIP_LAUNCH_BLOCKING=1 timeout -k 10 300 python -u tools/train_debug.py ${TD_CLIP:-train_tiny} > $OUT/train_debug.log 2>&1
      rc=$?; echo "tdebug rc=$rc"; tail -5 $OUT/train_debug.log; [ $rc -ne 0 ] && exit $rc ;;
    psnr)
      timeout -k 10 300 python -u tools/psnr_probe.py --seeds 3,5 > $OUT/psnr.log 2>&1
      rc=$?; tail -3 $OUT/psnr.log; [ $rc -ne 0 ] && exit $rc ;;
  esac
done
exit 0
