#!/bin/bash
# gffn at widths 128 / 64 (levels 2 / 1): the GoPro golden clips with gffn forced, the bf16 kernel-variant test,
# then the 1080p bench with and without it (top launch shapes)
set -o pipefail
TAG=${1:-g128}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_hip_parity.py -v --timeout 500 --timeout-method thread \
  -k "gffn_forced or (variants_agree and bf16)" > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|Error|gffn" $OUT/pytest.log | cut -c1-300 | tail -12; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-psnr --no-scaling-point --opt gffn_c64=1 --opt gffn_c128=1 > $OUT/bench_on.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-psnr --no-scaling-point --opt gffn_c128=1 > $OUT/bench_no64.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline --no-psnr --no-scaling-point > $OUT/bench_off.log 2>&1
rc=$?
for f in $OUT/bench_on.log $OUT/bench_no64.log $OUT/bench_off.log; do python3 - "$f" <<'PY'
import json, sys
for line in open(sys.argv[1]):
    if line.startswith("{"):
        d = json.loads(line)
        print(sys.argv[1], d["value"], d["ms_per_step"])
        top = d.get("top_launch_shapes_ms_per_step", {})
        for k in list(top)[:8]:
            print("   ", top[k], k)
PY
done
exit $rc
