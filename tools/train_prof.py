"""Attribute the training step's GPU time to torch ops and Python call sites (GPU box).

    python tools/train_prof.py [--batch 8] [--res 256] > gpurun_out/train_prof.txt

One warm-up step of bench.py --train's workload, then one step under torch.profiler: the top ops
by device time grouped by input shapes, and the top copy / cast ops grouped by their Python call
stack (where the layout conversions come from)."""
import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from turtlevsr_amd.synthetic import synthetic_frames, synthetic_state_dict  # noqa: E402
from turtlevsr_amd.train import Trainer, TurtleTrain  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--batch", type=int, default=8)
ap.add_argument("--res", type=int, default=256)
args = ap.parse_args()
dev = torch.device("cuda:0")
net = TurtleTrain(bench.load_opt())
shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
net.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(shapes, 0).items()})
net = net.to(dev).train()
tr = Trainer(net, amp="bf16")
B, R = args.batch, args.res
lq = torch.from_numpy(synthetic_frames((B, 5, 3, R, R), 1, name="lq")).to(dev)
gt = (lq + 0.05 * torch.from_numpy(synthetic_frames((B, 5, 3, R, R), 1, name="gt")).to(dev)).clamp(0, 1)
tr.train_step(lq, gt)
torch.cuda.synchronize()
acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
with torch.profiler.profile(activities=acts, record_shapes=True, with_stack=True) as prof:
    tr.train_step(lq, gt)
    torch.cuda.synchronize()
ka = prof.key_averages(group_by_input_shape=True)
print(ka.table(sort_by="self_device_time_total", row_limit=60, max_name_column_width=50, max_shapes_column_width=70))
# torch ops and autograd nodes outside the HIP op set (which ops the remaining ATen time belongs to)
ko = [e for e in prof.key_averages() if (e.key.startswith("aten::") or "Backward" in e.key) and not e.key.startswith("_")]
ko.sort(key=lambda e: -e.device_time_total)
print("\n==== torch ops / autograd nodes by device time (incl. children) ====")
for e in ko[:60]:
    print(f"{e.device_time_total / 1e3:9.2f} ms  n={e.count:5d}  {e.key}")
ks = prof.key_averages(group_by_stack_n=6)
rows = [e for e in ks if any(s in e.key for s in ("copy", "to", "contiguous", "clone", "cat", "permute"))]
rows.sort(key=lambda e: -e.self_device_time_total)
print("\n==== copy-like ops by call stack ====")
for e in rows[:30]:
    print(f"{e.self_device_time_total / 1e3:9.2f} ms  n={e.count:5d}  {e.key}")
    for s in e.stack[:6]:
        print("        ", s)
