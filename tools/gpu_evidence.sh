#!/bin/bash
# Round-end evidence on the final kernel sources (one gpurun call): the rocprofv3 kernel-trace
# summary of a short 1080p bench (trace kept in /tmp, only the stats CSV returned, stamped with the
# kernel source hash), then the PMC HBM-traffic passes (tools/gpu_pmc.sh -> pmc_traffic.json).
#   bash tools/gpu_evidence.sh <tag>
set -o pipefail
TAG=${1:-ev}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
HASH=$(python3 -c "import sys; sys.path.insert(0, '.'); from turtlevsr_amd import build; print(build.source_hash())")
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /tmp/ev_trace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-scaling-point > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; tail -1 $OUT/trace.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
f=$(find /tmp/ev_trace -name '*kernel_stats.csv' | head -1)
{ echo "# source_hash=$HASH (turtlevsr_amd/build.py source_hash), rocprofv3 --kernel-trace --stats, bench.py --steps 10 --warmup 3 (1080p bf16, 3 priming + 13 frames + the roofline pass)"; cat "$f"; } > $OUT/1080p_bf16_kernel_stats.csv
head -8 $OUT/1080p_bf16_kernel_stats.csv | cut -c1-160
bash tools/gpu_pmc.sh ${TAG}_pmc
