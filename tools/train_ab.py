"""A/B of the training step on one box: `python tools/train_ab.py [nocache]` runs bench.py --train
in-process, optionally with the shared-weight cast cache (train_ops._weight_cast) bypassed."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import turtlevsr_amd.train_ops as T  # noqa: E402

if len(sys.argv) > 1 and sys.argv[1] == "nocache":
    T._weight_cast = lambda w, gdt: (w.to(gdt).contiguous(), None)
sys.argv = ["bench.py", "--train", "--steps", "6", "--warmup", "2"]
import bench  # noqa: E402

bench.main()
