"""bench.py's workload selection (CPU only: argument resolution, no GPU call).

The driver runs `bench.py --gpus N --steps K --warmup W` with no other flags: N = 1 is the headline
configuration BASELINE.json's metric is quoted on (1920x1080, B = 1), N > 1 the north-star scaling
workload (synthetic 256x256 5-frame clips, 8 per GPU: "throughput on synthetic 256x256x5-frame
clips reported at 1/2/4/8 GPUs"), whose N = 1 point the default line carries."""
import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402


def test_default_single_gpu_line_is_the_1080p_headline():
    args, default_line = bench.parse_args(["--gpus", "1", "--steps", "5", "--warmup", "2"])
    assert (args.res, args.batch, args.graph, args.sr, args.train) == ("1080p", 1, False, False, False)
    assert bench.RES[args.res] == (1080, 1920)
    assert default_line


@pytest.mark.parametrize("n", [2, 4, 8])
def test_multi_gpu_default_is_the_256_clip_scaling_workload(n):
    args, default_line = bench.parse_args(["--gpus", str(n), "--steps", "5", "--warmup", "2"])
    assert bench.RES[args.res] == (256, 256)
    assert args.batch == bench.SCALE_BATCH == 8
    assert args.graph and args.no_roofline
    assert not default_line


def test_explicit_flags_win():
    args, default_line = bench.parse_args(["--gpus", "2", "--res", "1080p"])
    assert (args.res, args.batch, args.graph) == ("1080p", 1, False)
    args, default_line = bench.parse_args(["--res", "256", "--batch", "8"])
    assert not default_line and args.batch == 8
