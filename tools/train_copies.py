"""Where does the training graph copy / cast tensors? (CPU, no GPU needed)

    python tools/train_copies.py [--res 64] [--batch 1]

Runs one training step of the GoPro-width graph on CPU with an op set that mirrors HipOps' memory
formats (channels-last outputs, rows() re-layouts its inputs), under a TorchDispatchMode that logs
every copy-like aten op (copy_, _to_copy, clone, cat, zeros/fill) with its shape, dtype, strides
and the graph source line that issued it (forward) or the autograd node being run (backward).
Prints the totals by (site, op) sorted by bytes moved."""
import argparse
import collections
import os
import sys
import traceback

import torch
import torch.nn.functional as F
from torch.utils._python_dispatch import TorchDispatchMode

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
import bench  # noqa: E402
from turtlevsr_amd.synthetic import synthetic_frames, synthetic_state_dict  # noqa: E402
from turtlevsr_amd.train import TurtleTrain, Trainer  # noqa: E402

CL = torch.channels_last
NONCL = collections.Counter()


def rows(t):
    """train_ops.rows: NHWC pixel rows with channel stride 1 are taken as they are, else copied."""
    B, Cc, H, W = t.shape
    s = t.stride()
    ld = s[3] if W > 1 else (s[2] if H > 1 else (s[0] if B > 1 else Cc))
    ok = (Cc == 1 or s[1] == 1) and ld >= Cc and (W == 1 or s[3] == ld) and (H == 1 or s[2] == W * ld) and \
         (B == 1 or s[0] == H * W * ld)
    return t if ok else t.contiguous(memory_format=CL)


def _act(x):
    if torch.is_autocast_enabled("cpu") and x.dtype == torch.float32:
        return x.to(torch.get_autocast_dtype("cpu"))
    return x


class _Mimic(torch.autograd.Function):
    """y = f(rows(x)) as a channels-last output; backward re-layouts dy with rows() like HipOps."""

    @staticmethod
    def forward(ctx, x, fn, *params):
        ctx.fn, ctx.np = fn, len(params)
        xr = rows(x)
        ctx.save_for_backward(xr, *params)
        with torch.enable_grad():
            pass
        y = fn(xr.detach(), *[p.detach() for p in params])
        return y.contiguous(memory_format=CL)

    @staticmethod
    def backward(ctx, dy):
        xr, *params = ctx.saved_tensors
        if rows(dy) is not dy:
            NONCL[(getattr(ctx.fn, "__qualname__", "?").split(".")[1], tuple(dy.shape), tuple(dy.stride()), str(dy.dtype))] += 1
        dy = rows(dy.to(xr.dtype))
        with torch.enable_grad():
            xi = xr.detach().requires_grad_(True)
            ps = [p.detach().requires_grad_(p.requires_grad) for p in params]
            y = ctx.fn(xi, *ps)
        grads = torch.autograd.grad(y, [xi] + [p for p in ps if p.requires_grad], dy, allow_unused=True)
        gx, rest = grads[0], list(grads[1:])
        out = []
        for p in ps:
            out.append(rest.pop(0) if p.requires_grad else None)
        return (rows(gx) if gx is not None else None, None, *out)


def _ln(x, w, b, biasfree):
    xf = x.float()
    mu = xf.mean(1, keepdim=True)
    var = ((xf - mu) ** 2).mean(1, keepdim=True)
    y = (xf if biasfree else xf - mu) / torch.sqrt(var + 1e-5) * w.view(1, -1, 1, 1)
    return (y if biasfree or b is None else y + b.view(1, -1, 1, 1)).to(x.dtype)


class MimicOps:
    channels_last = True

    @staticmethod
    def layer_norm(x, w, b, biasfree):
        ps = (w,) if b is None else (w, b)
        od = _act(x[:, :1, :1, :1]).dtype                # HipOps: fp32 x is read as is, y in the autocast dtype
        return _Mimic.apply(x, lambda t, *p: _ln(t, p[0], p[1] if len(p) > 1 else None, biasfree).to(od), *ps)

    @staticmethod
    def dwconv3x3(x, w, b):
        if b is None:
            return _Mimic.apply(_act(x), lambda t, ww: F.conv2d(t, ww.to(t.dtype), None, 1, 1, 1, t.shape[1]), w)
        return _Mimic.apply(_act(x), lambda t, ww, bb: F.conv2d(t, ww.to(t.dtype), bb.to(t.dtype), 1, 1, 1, t.shape[1]), w, b)

    @staticmethod
    def gelu_gate(x):
        return _Mimic.apply(_act(x), lambda t: F.gelu(t[:, :t.shape[1] // 2]) * t[:, t.shape[1] // 2:])

    @staticmethod
    def conv1x1(x, w, b):
        x = _act(x)
        if w.dim() == 4:
            w = w.reshape(w.shape[0], w.shape[1])
        if w.dim() == 2:
            fn = (lambda t, ww, bb: torch.einsum("bkhw,nk->bnhw", t, ww.to(t.dtype)) + bb.to(t.dtype).view(1, -1, 1, 1)) \
                if b is not None else (lambda t, ww: torch.einsum("bkhw,nk->bnhw", t, ww.to(t.dtype)))
        else:
            fn = (lambda t, ww, bb: torch.einsum("bkhw,bnk->bnhw", t, ww.to(t.dtype)) + bb.to(t.dtype).view(1, -1, 1, 1)) \
                if b is not None else (lambda t, ww: torch.einsum("bkhw,bnk->bnhw", t, ww.to(t.dtype)))
        return _Mimic.apply(x, fn, *((w, b) if b is not None else (w,)))

    @staticmethod
    def gelu(x):
        return _Mimic.apply(_act(x), lambda t: F.gelu(t))

    @staticmethod
    def window_conv(x, w, b, ws):
        if b is None:
            return _Mimic.apply(_act(x), lambda t, ww: F.conv2d(t, ww.to(t.dtype), None, ws, 1, 1, t.shape[1]), w)
        return _Mimic.apply(_act(x), lambda t, ww, bb: F.conv2d(t, ww.to(t.dtype), bb.to(t.dtype), ws, 1, 1, t.shape[1]), w, b)

    @staticmethod
    def conv3x3(x, w, b=None):
        return _Mimic.apply(_act(x), lambda t, ww: F.conv2d(t, ww.to(t.dtype), None, 1, 1), w)

    @staticmethod
    def norm_gram(qk, heads, sink=None):
        qk = rows(_act(qk))
        b, c2, h, w = qk.shape
        c = c2 // 2
        qh = qk[:, :c].reshape(b, heads, c // heads, h * w).float()
        kh = qk[:, c:].reshape(b, heads, c // heads, h * w).float()
        qh = qh / qh.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        kh = kh / kh.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        return qh @ kh.transpose(-2, -1)

    @staticmethod
    def gram(q, k, heads):
        q, k = rows(_act(q)), rows(_act(k))
        b, c, h, w = q.shape
        qh, kh = q.reshape(b, heads, c // heads, h * w), k.reshape(b, heads, c // heads, h * w)
        return (qh.float() @ kh.float().transpose(-2, -1))


COPY_OPS = ("copy_", "_to_copy", "clone", "cat", "zeros", "fill_", "new_zeros", "zero_", "slice_backward", "contiguous")


class CopyLog(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.tot = collections.Counter()
        self.n = collections.Counter()
        self.phase = "fwd"

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.__name__ if hasattr(func, "__name__") else str(func)
        if any(name.startswith(s) for s in COPY_OPS):
            t = out if torch.is_tensor(out) else (args[0] if args and torch.is_tensor(args[0]) else None)
            if t is not None:
                site = "?"
                stack = list(reversed(traceback.extract_stack()[:-1]))
                for i, fr in enumerate(stack):
                    if "turtlevsr_amd" in fr.filename or "train_copies" in fr.filename:
                        site = f"{os.path.basename(fr.filename)}:{fr.lineno} {fr.line.strip()[:70]}"
                        if fr.filename.endswith("train_ops.py"):     # name the graph line that called the op
                            up = next((g for g in stack[i + 1:] if g.filename.endswith("train.py")), None)
                            if up is not None:
                                site += f"  <- train.py:{up.lineno} {up.line.strip()[:50]}"
                        break
                node = torch._C._current_autograd_node()
                if node is not None:
                    site = f"[bwd {node.name()}] " + site
                src = args[1] if name.startswith("copy_") and len(args) > 1 and torch.is_tensor(args[1]) else None
                desc = f"{name} {tuple(t.shape)} {str(t.dtype)[6:]}"
                if name.startswith("clone") and args and torch.is_tensor(args[0]):
                    a0 = args[0]
                    desc += f" <- {str(a0.dtype)[6:]} cl={a0.is_contiguous(memory_format=CL)} nchw={a0.is_contiguous()} stride={a0.stride()}"
                if src is not None:
                    desc += f" <- {str(src.dtype)[6:]} cl={src.is_contiguous(memory_format=CL)} nchw={src.is_contiguous()}"
                key = (self.phase, site, desc.split(" (")[0] + (" " + desc.split(" <- ")[1] if " <- " in desc else "")
                       + (f" {tuple(t.shape)}" if "train.py:146" in site else ""))
                self.tot[key] += t.numel() * t.element_size()
                self.n[key] += 1
        return out


ap = argparse.ArgumentParser()
ap.add_argument("--res", type=int, default=64)
ap.add_argument("--batch", type=int, default=1)
ap.add_argument("--frames", type=int, default=2)
ap.add_argument("--gpu", action="store_true", help="the real HipOps on cuda:0 (backward on this thread)")
args = ap.parse_args()
torch.manual_seed(0)
dev = "cuda" if args.gpu else "cpu"
if args.gpu:
    torch.autograd.set_multithreading_enabled(False)
net = TurtleTrain(bench.load_opt(), ops=None if args.gpu else MimicOps)
shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
net.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(shapes, 0).items()})
net = net.to(dev).train()
B, R, T = args.batch, args.res, args.frames
lq = torch.from_numpy(synthetic_frames((B, T, 3, R, R), 1, name="lq")).to(dev)
gt = lq.clone()
log = CopyLog()
with log:
    with torch.autocast(dev, dtype=torch.bfloat16):
        kc = vc = None
        total = 0.0
        for j in range(T):
            inp = torch.stack([lq[:, j if j == 0 else j - 1], lq[:, j]], dim=1)
            out, kc, vc = net(inp, kc, vc)
            total = total + F.l1_loss(out.float(), gt[:, j].float())
    loss = total / T + 0 * sum(p.sum() for p in net.parameters())
    log.phase = "bwd"
    loss.backward()
rows_ = sorted(log.tot.items(), key=lambda kv: -kv[1])
print(f"{'MB':>9} {'n':>5}  phase  site / op")
for (ph, site, desc), by in rows_[:70]:
    print(f"{by / 1e6:9.2f} {log.n[(ph, site, desc)]:5d}  {ph}  {site}  ::  {desc}")
print("total MB", sum(log.tot.values()) / 1e6)
for k, v in NONCL.most_common(30):
    print("non-CL dy", v, k)
