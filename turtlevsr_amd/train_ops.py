"""Autograd Functions over the hand-written HIP training kernels (include/turtle_train.h).

The training graph (turtlevsr_amd/train.py) runs these three op families through libturtle_hip.so,
forward and backward:

* ``layer_norm``  per-pixel LayerNorm over channels (turtle_t1_arch.py:67-112), 98 per frame;
* ``dwconv3x3``   depthwise 3x3 / pad 1 convolutions (99 per frame: qkv_dwconv, conv2, dwconv,
                  qk/v/kv_dwconv);
* ``gelu_gate``   gelu(x1) * x2 of the GatedFeedForward (turtle_t1_arch.py:176).

They run on the caller's current HIP stream; weights and their gradients are fp32, activations
fp32 or bf16 (autocast). There is no CPU path: a CPU tensor or a missing library raises.
"""
from __future__ import annotations

import ctypes as C

import torch

from . import _lib

_train = None


def lib():
    global _train
    if _train is not None:
        return _train
    L = _lib.lib()
    vp, i64, ci = C.c_void_p, C.c_int64, C.c_int
    L.turtle_train_ln_fwd.argtypes = [vp, vp, vp, vp, vp, vp, i64, ci, i64, ci, ci, vp]
    L.turtle_train_ln_bwd.argtypes = [vp, vp, vp, vp, vp, vp, vp, vp, i64, ci, i64, ci, ci, vp]
    L.turtle_train_dw3x3_fwd.argtypes = [vp, vp, vp, vp, i64, ci, ci, ci, ci, ci, vp]
    L.turtle_train_dw3x3_wgrad.argtypes = [vp, vp, vp, vp, i64, ci, ci, ci, ci, vp]
    L.turtle_train_gate_fwd.argtypes = [vp, vp, i64, ci, i64, ci, vp]
    L.turtle_train_gate_bwd.argtypes = [vp, vp, vp, i64, ci, i64, ci, vp]
    _train = L
    return L


def _p(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _dt(t: torch.Tensor) -> int:
    if t.dtype == torch.float32:
        return 0
    if t.dtype == torch.bfloat16:
        return 1
    raise TypeError(f"training kernels take fp32 / bf16 activations, got {t.dtype}")


def _stream(t):
    if t.device.type != "cuda":
        raise RuntimeError("turtle training kernels run on a ROCm device only")
    return C.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def _check(rc, what):
    if rc != 0:
        raise RuntimeError(f"{what} failed ({rc})")


class _LayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b, biasfree: bool):
        x = x.contiguous()
        N, Cc = x.shape[0], x.shape[1]
        HW = x[0, 0].numel()
        y = torch.empty_like(x)
        mu = torch.empty(N * HW, dtype=torch.float32, device=x.device)
        rs = torch.empty_like(mu)
        w32 = w.float().contiguous()
        b32 = None if b is None else b.float().contiguous()
        _check(lib().turtle_train_ln_fwd(_p(x), _p(w32), _p(b32), _p(y), _p(mu), _p(rs), N, Cc, HW, int(biasfree), _dt(x),
                                         _stream(x)), "ln_fwd")
        ctx.save_for_backward(x, w32, mu, rs)
        ctx.biasfree, ctx.has_b = biasfree, b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w32, mu, rs = ctx.saved_tensors
        dy = dy.contiguous().to(x.dtype)
        N, Cc = x.shape[0], x.shape[1]
        HW = x[0, 0].numel()
        dx = torch.empty_like(x)
        dw = torch.zeros(Cc, dtype=torch.float32, device=x.device)
        db = torch.zeros(Cc, dtype=torch.float32, device=x.device) if ctx.has_b else None
        _check(lib().turtle_train_ln_bwd(_p(x), _p(w32), _p(mu), _p(rs), _p(dy), _p(dx), _p(dw), _p(db), N, Cc, HW,
                                         int(ctx.biasfree), _dt(x), _stream(x)), "ln_bwd")
        return dx, dw, db, None


class _DWConv(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w, b):
        x = x.contiguous()
        N, Cc, H, W = x.shape
        w32 = w.float().reshape(Cc, 9).contiguous()
        b32 = None if b is None else b.float().contiguous()
        y = torch.empty_like(x)
        _check(lib().turtle_train_dw3x3_fwd(_p(x), _p(w32), _p(b32), _p(y), N, Cc, H, W, 0, _dt(x), _stream(x)), "dw_fwd")
        ctx.save_for_backward(x, w32)
        ctx.has_b = b is not None
        return y

    @staticmethod
    def backward(ctx, dy):
        x, w32 = ctx.saved_tensors
        dy = dy.contiguous().to(x.dtype)
        N, Cc, H, W = x.shape
        dx = torch.empty_like(x)
        st = _stream(x)
        _check(lib().turtle_train_dw3x3_fwd(_p(dy), _p(w32), None, _p(dx), N, Cc, H, W, 1, _dt(x), st), "dw_dgrad")
        dw = torch.zeros(Cc, 9, dtype=torch.float32, device=x.device)
        db = torch.zeros(Cc, dtype=torch.float32, device=x.device) if ctx.has_b else None
        _check(lib().turtle_train_dw3x3_wgrad(_p(x), _p(dy), _p(dw), _p(db), N, Cc, H, W, _dt(x), st), "dw_wgrad")
        return dx, dw.reshape(Cc, 1, 3, 3), db


class _Gate(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        x = x.contiguous()
        N, C2 = x.shape[0], x.shape[1]
        h, HW = C2 // 2, x[0, 0].numel()
        y = torch.empty((N, h) + tuple(x.shape[2:]), dtype=x.dtype, device=x.device)
        _check(lib().turtle_train_gate_fwd(_p(x), _p(y), N, h, HW, _dt(x), _stream(x)), "gate_fwd")
        ctx.save_for_backward(x)
        return y

    @staticmethod
    def backward(ctx, dy):
        (x,) = ctx.saved_tensors
        dy = dy.contiguous().to(x.dtype)
        N, C2 = x.shape[0], x.shape[1]
        dx = torch.empty_like(x)
        _check(lib().turtle_train_gate_bwd(_p(x), _p(dy), _p(dx), N, C2 // 2, x[0, 0].numel(), _dt(x), _stream(x)), "gate_bwd")
        return dx


def _act(x: torch.Tensor) -> torch.Tensor:
    """Activations enter the kernels in the autocast dtype (bf16 under bf16 autocast)."""
    if torch.is_autocast_enabled("cuda") and x.dtype == torch.float32:
        return x.to(torch.get_autocast_dtype("cuda"))
    return x


class HipOps:
    """The op set of the training graph, on the HIP kernels."""

    @staticmethod
    def layer_norm(x, w, b, biasfree: bool):
        return _LayerNorm.apply(_act(x), w, b, biasfree)

    @staticmethod
    def dwconv3x3(x, w, b):
        return _DWConv.apply(_act(x), w, b)

    @staticmethod
    def gelu_gate(x):
        return _Gate.apply(_act(x))
