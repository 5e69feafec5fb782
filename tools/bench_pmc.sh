#!/bin/bash
# SQ / HBM counter passes over short 1080p bench runs, restricted to kernels matching a regex
# (GPU box): bash tools/bench_pmc.sh <tag> <kernel-regex>
# One rocprofv3 --pmc pass per counter group (separate runs: counters are not split over passes).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/${1:-bpmc}; K=${2:-fused2_kernel}
mkdir -p $OUT
B="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-psnr --no-scaling-point --no-roofline"
timeout -s KILL 150 rocprofv3 --kernel-include-regex "$K" --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES -f csv -d $OUT/p1 -o run -- $B > $OUT/p1.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --kernel-include-regex "$K" --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_MISC -f csv -d $OUT/p2 -o run -- $B > $OUT/p2.log 2>&1 &&
timeout -s KILL 150 rocprofv3 --kernel-include-regex "$K" --pmc SQ_ACTIVE_INST_MFMA SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_WAIT_INST_VMEM SQ_INSTS_VMEM -f csv -d $OUT/p3 -o run -- $B > $OUT/p3.log 2>&1
rc=$?; echo "bench_pmc rc=$rc"; exit $rc
