#!/bin/bash
# attn_fin A/B (one gpurun call): variant / parity tests, then 256x256 B = 1 / B = 8 graph and 1080p eager lines per setting
set -o pipefail
TAG=${1:-attnfin}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "variants or clip_bf16 or clip_fp32 or repeatable" > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
OPTSETS="attn_fin=0;attn_fin=1" bash tools/gpu_small_ab.sh $TAG || exit 1
for o in 0 1; do
  timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-psnr --no-scaling-point --warmup 3 --opt attn_fin=$o > $OUT/b1080_$o.log 2>&1 || exit 1
  echo "[attn_fin=$o] 1080p $(tail -1 $OUT/b1080_$o.log | cut -c1-120)"
done
