#!/bin/bash
# 1080p bench under several environment settings (one gpurun call); per setting the frame time and
# the summed time of the launch shapes matching a regex. Outputs under gpurun_out/<tag>/.
#   bash tools/gpu_sweep_env.sh <tag> '<shape regex>' VAR=V1 VAR=V2 ...
set -o pipefail
TAG=$1; RE=$2; shift 2
mkdir -p gpurun_out/$TAG
export TMPDIR=/tmp
i=0
for KV in base "$@"; do
  i=$((i + 1))
  if [ "$KV" = base ]; then E=(); else E=("$KV"); fi
  env "${E[@]}" TURTLE_BENCH_DUMP=gpurun_out/$TAG/$i.tsv timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-psnr --warmup 3 > gpurun_out/$TAG/$i.log 2>&1
  rc=$?; [ $rc -ne 0 ] && { echo "$KV failed rc=$rc"; exit $rc; }
  python3 tools/launch_report.py gpurun_out/$TAG/$i.tsv --steps 3 --top 200 > gpurun_out/$TAG/$i.txt
  echo "$KV: $(head -1 gpurun_out/$TAG/$i.txt) | matched $(grep -E "$RE" gpurun_out/$TAG/$i.txt | awk '{s+=$1} END {print s}') ms"
done
