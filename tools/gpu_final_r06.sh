#!/bin/bash
# Round-6 end evidence on the final sources (one gpurun call): smoke(); PMC HBM traffic passes
# (tools/gpu_pmc.sh) copied to profiles/pmc_traffic.json so the bench line below carries `traffic`;
# the rocprofv3 kernel-trace stats (tools/gpu_evidence.sh minus PMC); the default bench line
# (1080p, CPU baseline, PSNR, oracle pin, scaling point).
#   bash tools/gpu_final_r06.sh <tag>
set -o pipefail
TAG=${1:-r06z}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -2 $OUT/smoke.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_pmc.sh ${TAG}_pmc > $OUT/pmc.log 2>&1
rc=$?; echo "pmc rc=$rc"; tail -3 $OUT/pmc.log | cut -c1-300; [ $rc -ne 0 ] && exit $rc
cp gpurun_out/${TAG}_pmc/pmc_traffic.json profiles/pmc_traffic.json
HASH=$(python3 -c "import sys; sys.path.insert(0, '.'); from turtlevsr_amd import build; print(build.source_hash())")
timeout -k 10 400 rocprofv3 --kernel-trace --stats -f csv -d /tmp/ev_trace -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-psnr --no-scaling-point > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -ne 0 ] && exit $rc
f=$(find /tmp/ev_trace -name '*kernel_stats.csv' | head -1)
{ echo "# source_hash=$HASH (turtlevsr_amd/build.py source_hash), rocprofv3 --kernel-trace --stats, bench.py --steps 10 --warmup 3 (1080p bf16, 3 priming + 13 frames + the roofline pass)"; cat "$f"; } > $OUT/1080p_bf16_kernel_stats.csv
head -6 $OUT/1080p_bf16_kernel_stats.csv | cut -c1-160
timeout -k 10 900 python -u bench.py > $OUT/bench_1080p.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 $OUT/bench_1080p.log | cut -c1-800; exit $rc
