"""Which call sites issue the training step's ATen memory ops? (GPU box)

    python tools/train_sites.py [--batch 8] [--res 256] [--frames 5] > out.txt

One Trainer step of the GoPro network (bf16 autocast, HIP op set) under a TorchDispatchMode that logs
every copy / cast / cat / fill / elementwise-add / reduction aten op with the innermost
turtlevsr_amd (or torch.autograd) source line on the Python stack - the autograd engine's own ops
(gradient accumulation of a parameter used by several frames, view backward) have none and are
listed as <engine>. Prints launches and bytes by (site, op), sorted by bytes."""
import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import bench  # noqa: E402
from turtlevsr_amd.synthetic import synthetic_frames, synthetic_state_dict  # noqa: E402
from turtlevsr_amd.train import Trainer, TurtleTrain  # noqa: E402

WATCH = ("copy_", "_to_copy", "clone", "cat", "fill_", "zero_", "zeros", "add", "add_", "sum", "mul", "sub", "div",
         "new_zeros", "index", "stack", "masked_fill", "where", "neg", "expand", "contiguous")


def _site():
    fr_in = [fr for fr in reversed(traceback.extract_stack()[:-3])
             if "turtlevsr_amd" in fr.filename or ("tools" in fr.filename and "train_sites" not in fr.filename)]
    if fr_in:
        return " < ".join(f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.name}" for fr in fr_in[:2])
    node = torch._C._current_autograd_node()       # the backward node the engine is running (or None)
    if node is None:
        return "<engine>"
    where = ""
    try:                                            # anomaly mode keeps the node's forward stack
        tb = node.metadata.get("traceback_")
        if tb:
            lines = [ln for ln in "".join(tb).splitlines() if "turtlevsr_amd" in ln and "File" in ln]
            if lines:
                ln = lines[-1].strip()
                f = ln.split('"')[1]
                where = f" fwd {os.path.basename(f)}:{ln.split('line ')[1].split(',')[0]}"
    except Exception:                               # noqa: BLE001 - attribution only
        pass
    return f"<engine: {node.name()}{where}>"


class Log(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.n = collections.Counter()
        self.b = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.overloadpacket.__name__
        if name in WATCH:
            t = out if isinstance(out, torch.Tensor) else None
            if t is not None and t.is_cuda:
                key = (_site(), name, str(t.dtype).replace("torch.", ""))
                self.n[key] += 1
                self.b[key] += t.numel() * t.element_size()
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--res", type=int, default=256)
    ap.add_argument("--frames", type=int, default=5)
    ap.add_argument("--no-acc", action="store_true", help="autograd's per-use parameter gradients (no accumulator)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    opt = bench.load_opt()
    net = TurtleTrain(opt)
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(shapes, 0).items()})
    net = net.to(dev).train()
    tr = Trainer(net, amp="bf16", accumulate_grads=not a.no_acc)
    lq = torch.from_numpy(synthetic_frames((a.batch, a.frames, 3, a.res, a.res), 1, name="lq")).to(dev)
    gt = torch.from_numpy(synthetic_frames((a.batch, a.frames, 3, a.res, a.res), 1, name="gt")).to(dev)
    tr.train_step(lq, gt)                                       # warm caches (weight casts, workspaces)
    torch.cuda.synchronize()
    log = Log()
    with torch.autograd.set_detect_anomaly(True, check_nan=False), log:
        tr.train_step(lq, gt)
    torch.cuda.synchronize()
    tot_n, tot_b = sum(log.n.values()), sum(log.b.values())
    print(f"one step, batch {a.batch} x {a.frames} frames at {a.res}^2: {tot_n} logged aten ops, {tot_b / 1e9:.2f} GB of outputs")
    print(f"{'launches':>9} {'GB out':>8}  op/dtype  site")
    for key in sorted(log.b, key=lambda k: -log.b[k])[:80]:
        print(f"{log.n[key]:9d} {log.b[key] / 1e9:8.3f}  {key[1]}/{key[2]}  {key[0]}")
    print("\nby op:")
    byop_n, byop_b = collections.Counter(), collections.Counter()
    for k in log.n:
        byop_n[k[1]] += log.n[k]
        byop_b[k[1]] += log.b[k]
    for k in sorted(byop_b, key=lambda k: -byop_b[k]):
        print(f"{byop_n[k]:9d} {byop_b[k] / 1e9:8.3f}  {k}")


if __name__ == "__main__":
    main()
