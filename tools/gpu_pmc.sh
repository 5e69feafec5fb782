#!/bin/bash
# PMC HBM traffic of the dominant launch shapes on the current build (one gpurun call): separate
# FETCH_SIZE / WRITE_SIZE passes over a short 1080p bench, then tools/pmc_traffic.py ->
# gpurun_out/<tag>/pmc_traffic.json (copy to profiles/pmc_traffic.json; it carries the kernel source hash).
set -o pipefail
TAG=${1:-pmc}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# 1080p frames only (no 256x256 scaling point: persistent kernels have the same grid at every size)
BENCH="bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-psnr --no-scaling-point --no-roofline"
KRE='gffn_kernel|dwgemm_kernel|ffn_kernel|fused2_kernel|dw_rows_kernel|gemm_pn_kernel|tilepd_kernel'
timeout -s KILL 400 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT/fetch -o run -- python3 $BENCH > $OUT/fetch.log 2>&1 &&
timeout -s KILL 400 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$KRE" -f csv -d $OUT/write -o run -- python3 $BENCH > $OUT/write.log 2>&1
rc=$?; echo "pmc rc=$rc"; [ $rc -ne 0 ] && exit $rc
python3 tools/pmc_traffic.py $OUT \
  'gffn nimg=1 H=272 W=480 hd=640@@gffn_kernel<256, 0>' \
  'gffn nimg=1 H=544 W=960 C=128 hd=320@@gffn_kernel<128, 0>' \
  'dwgemm gate=1 nimg=1 H=272 W=480 K=640 N=256@@dwgemm_kernel<2>' \
  'tilepd mode=0 nimg=1 H=272 W=480 C=256 N1=768@@tilepd_kernel<0,' \
  'ffn M=522240 C=128@@ffn_kernel<128>' \
  'ffn M=2088960 C=64@@ffn_kernel<64>' \
  'fused2 mode=2 nimg=1 H=1088 W=1920 C=64 N1=320 N2=64 ln=1 ndst=0@@fused2_kernel<2, 64,' \
  'fused2 mode=1 nimg=1 H=1088 W=1920 C=64 N1=128 N2=64 ln=1 ndst=0@@fused2_kernel<1, 64,' \
  'fused2 mode=1 nimg=1 H=544 W=960 C=128 N1=256 N2=128 ln=1 ndst=0@@fused2_kernel<1, 128,' \
  > $OUT/pmc_traffic.json
rc=$?; python3 -c "import json; d=json.load(open('$OUT/pmc_traffic.json')); print(d['source_hash'], json.dumps(d['per_tag'], indent=0)[:1500])"; exit $rc
