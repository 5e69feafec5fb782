#!/bin/bash
# One training-kernel iteration on a GPU box: the op-level GPU training tests, then the kernel stats
# of a 3-step config-5 bench (tools/gpu_train_prof_r06.sh).
set -o pipefail
TAG=${1:-ti}
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -u -m pytest tests/test_train.py -m gpu -x -v --timeout 300 --timeout-method thread \
  -k "ops_match or fused_residual or gelu_window or matches_reference_gradients or config5" > gpurun_out/$TAG/pytest.log 2>&1
rc=$?; tail -3 gpurun_out/$TAG/pytest.log; [ $rc -ne 0 ] && exit $rc
bash tools/gpu_train_prof_r06.sh $TAG
