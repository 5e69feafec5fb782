"""Test infrastructure: the training graph's op set (layer_norm, dwconv3x3, gelu_gate) as plain
torch ops, so the distributed trainer logic (DDP, BPTT, AdamW, loss reduction) can run in gloo
processes on CPU. The product op set is turtlevsr_amd.train_ops.HipOps (HIP kernels, no CPU path);
tests/test_train.py checks both against the reference's own gradients."""
import torch
import torch.nn.functional as F


class AtenOps:
    channels_last = False
    @staticmethod
    def layer_norm(x, w, b, biasfree):
        mu = x.mean(dim=1, keepdim=True)
        var = ((x - mu) ** 2).mean(dim=1, keepdim=True)
        if biasfree:
            return x / torch.sqrt(var + 1e-5) * w.view(1, -1, 1, 1)
        return (x - mu) / torch.sqrt(var + 1e-5) * w.view(1, -1, 1, 1) + b.view(1, -1, 1, 1)

    @staticmethod
    def dwconv3x3(x, w, b):
        return F.conv2d(x, w, b, 1, 1, 1, x.shape[1])

    @staticmethod
    def gelu_gate(x):
        h = x.shape[1] // 2
        return F.gelu(x[:, :h]) * x[:, h:]

    @staticmethod
    def conv1x1(x, w, b):
        if w.dim() == 4:
            return F.conv2d(x, w, b)
        if w.dim() == 2:                                # [N, K]: one shared weight set
            return F.conv2d(x, w[:, :, None, None], b)
        y = torch.einsum("bkhw,bnk->bnhw", x, w)        # one weight set per image
        return y if b is None else y + b.view(1, -1, 1, 1)

    @staticmethod
    def gram(q, k, heads):
        b, c, h, w = q.shape
        qh, kh = q.reshape(b, heads, c // heads, h * w), k.reshape(b, heads, c // heads, h * w)
        return qh @ kh.transpose(-2, -1)

    @staticmethod
    def norm_gram(qk, heads):
        b, c2, h, w = qk.shape
        c = c2 // 2
        q, k = qk[:, :c].reshape(b, heads, c // heads, h * w), qk[:, c:].reshape(b, heads, c // heads, h * w)
        q = q / q.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        k = k / k.norm(dim=-1, keepdim=True).clamp_min(1e-12)
        return q @ k.transpose(-2, -1)
