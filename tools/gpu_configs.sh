set -o pipefail
mkdir -p gpurun_out/cfg
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_hip_configs.py -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/cfg/t.log 2>&1
rc=$?; tail -6 gpurun_out/cfg/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u bench.py --res 256 --no-cpu-baseline > gpurun_out/cfg/b256.log 2>&1 && tail -1 gpurun_out/cfg/b256.log &&
timeout -k 10 200 python -u bench.py --res 256 --batch 8 --no-cpu-baseline > gpurun_out/cfg/b256x8.log 2>&1 && tail -1 gpurun_out/cfg/b256x8.log &&
timeout -k 10 300 python -u bench.py --sr --no-cpu-baseline > gpurun_out/cfg/bsr.log 2>&1 && tail -1 gpurun_out/cfg/bsr.log
