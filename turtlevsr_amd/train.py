"""Training step of Turtle (BASELINE config 5): BPTT over the causal frame loop, AdamW, DDP over RCCL.

Restates the reference's training semantics (basicsr/models/video_restoration_model.py:26-108,
base_model.py:340-365, dist_util.py:15-30) on the GPU:

* ``TurtleTrain`` is the differentiable Turtle_t1 graph over the SAME parameter tree as the
  inference module (633 keys, turtlevsr_amd/params.py), so checkpoints move between training and
  the HIP inference path unchanged. On the GPU its LayerNorms, depthwise 3x3 convolutions, GELU
  gates and plain GELUs, pointwise 1x1 convolutions (forward, input and weight gradients), the
  channel-attention Gram, the Down / Upsample 3x3 convolutions and the SAB window convolutions run on
  hand-written HIP kernels with hand-written backward (``train_ops.HipOps``, include/turtle_train.h),
  on channels-last activations, and so do (round 5) the stem / ending convolutions, the FHR / CHM
  attention with its caches (per-channel L2 normalisation, cross-Gram, W_eff over the history) and the
  SAB core (scores, top-5 + L1-ball clipped softmax, A.v) up to SAB_MAX_KEYS keys per frame; what is
  left in torch is reshapes, concatenations and the ATen op set that the CPU tests differentiate.
* caches are NOT detached between frames: the loss of frame j back-propagates into frames < j
  through the history state (video_restoration_model.py:85-95);
* ``Trainer.train_step``: zero_grad -> autocast forward over the T frames -> L1 per frame summed,
  / T -> ``+ 0 * sum(p.sum())`` (every parameter in the graph, so DDP needs no unused-parameter
  search, :99) -> (GradScaler for fp16) backward -> AdamW step -> loss reduced to rank 0 (dist.reduce
  + / world_size, base_model.py:340-365). On the HIP op set (round 6) the weight gradients of the T
  frames accumulate in place into one fp32 arena (``train_ops.ParamGradAccumulator``; the 0 * sum(p)
  term then adds its zero gradient only to parameters no HIP op reported) and every block's
  residual add is the last GEMM's epilogue, its gradient summed inside the LayerNorm backward
  (``_ln_res``);
* multi-GPU: one process per GPU, ``torch.nn.parallel.DistributedDataParallel`` over the
  ``nccl`` backend (RCCL over xGMI on MI355X): the gradient all-reduce is bucketed and overlaps the
  backward; buckets are sized for xGMI (fewer, larger all-reduces of the 236 MB fp32 gradient).
"""
from __future__ import annotations

import math
import os
from typing import List, Optional

import torch
import torch.distributed as dist
import torch.nn.functional as F

from .params import TurtleParams

LN_EPS = 1e-5
_ATEN_SAB = os.environ.get("TURTLE_TRAIN_ATEN_SAB") == "1"     # A/B only: the SAB softmax chain as torch ops
L2_EPS = 1e-12
SAB_TOPK = 5
SAB_RADIUS = 4


def _l2n(x, dim):
    return x / x.norm(dim=dim, keepdim=True).clamp_min(L2_EPS)


def _act_dt(t: torch.Tensor) -> torch.dtype:
    """The dtype the attention finalize hands its per-image weight set to the HIP conv1x1 in: fp32 - the
    conv casts it to its GEMM dtype once (train_ops._weight_cast), its weight gradient comes back in
    fp32 (the reduction GEMM's output) and the finalize's backward needs no cast either way."""
    return torch.float32


def _res(res):
    """The residual keyword for an op set's conv1x1 (absent when there is none: ATen op sets)."""
    return {} if res is None else {"res": res}


def _plus(res, a):
    return a if res is None else res + a


def _conv1(m, x):
    return F.conv2d(x, m.weight, m.bias)


class _ChanSplit(torch.autograd.Function):
    """x[:, a:b] channel slices whose backward assembles the slice gradients in x's memory
    format. Plain slicing's backward (slice_backward) builds each slice gradient into a zero-filled
    NCHW tensor and sums them: three fills, three transposing copies and a re-layout back to
    channels-last per qkv split on the HIP graph (the largest copy traffic of the training step)."""

    @staticmethod
    def forward(ctx, x, sink, *sizes):
        ctx.sizes, ctx.sink = sizes, sink
        ctx.cl = x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last)
        outs, a = [], 0
        for n in sizes:
            outs.append(x.narrow(1, a, n))
            a += n
        return tuple(outs)

    @staticmethod
    def backward(ctx, *grads):
        if ctx.sink is not None:        # the consumers wrote their gradients into one buffer
            buf = ctx.sink.take(grads, ctx.sizes)
            if buf is not None:
                return (buf, None) + (None,) * len(ctx.sizes)
        ref = next(t for t in grads if t is not None)
        if ctx.cl:
            # each slice gradient copied once, in whatever layout it arrives, straight into its
            # channel range of the channels-last result (not re-laid out first, then concatenated)
            shape = list(ref.shape)
            shape[1] = sum(ctx.sizes)
            out = torch.empty(shape, dtype=ref.dtype, device=ref.device, memory_format=torch.channels_last)
            a = 0
            for g, n in zip(grads, ctx.sizes):
                if g is None:
                    out.narrow(1, a, n).zero_()
                else:
                    out.narrow(1, a, n).copy_(g)
                a += n
            return (out, None) + (None,) * len(ctx.sizes)
        parts = []
        for g, n in zip(grads, ctx.sizes):
            if g is None:
                shape = list(ref.shape)
                shape[1] = n
                g = torch.zeros(shape, dtype=ref.dtype, device=ref.device)
            parts.append(g)
        out = torch.cat(parts, dim=1)
        return (out, None) + (None,) * len(ctx.sizes)


def _split(x, *sizes, sink=None):
    return _ChanSplit.apply(x, sink, *sizes)


# the HIP SAB kernels take at most this many keys per frame (train_ops.hip: one wave per score row);
# larger token grids (training crops above ~512 x 512) go through the ATen top-5 / softmax chain
SAB_MAX_KEYS = 1024


def _sab_hip_ok(ops, name: str, n: int, g: int = 8, d: int = 8) -> bool:
    """Whether the StateAlignBlock core runs on the op set's HIP kernel `name` ('sab_attention' or
    'sab_softmax') for n keys of width g and value width d (n > 1024 used to raise)."""
    if not hasattr(ops, name) or _ATEN_SAB or n > SAB_MAX_KEYS:
        return False
    return name != "sab_attention" or (n % 8 == 0 and g % 8 == 0 and d % 8 == 0)


class _ToNCHW(torch.autograd.Function):
    """x.contiguous() for F.conv2d's NCHW path (a channels-last op set without a dense-conv kernel
    for that shape) whose gradient goes back in x's own memory format: otherwise the NCHW input
    gradient of the dense conv makes the channels-last residual-stream backward NCHW, and each
    following op re-lays it out."""

    @staticmethod
    def forward(ctx, x):
        ctx.cl = x.dim() == 4 and not x.is_contiguous() and x.is_contiguous(memory_format=torch.channels_last)
        return x.contiguous()

    @staticmethod
    def backward(ctx, g):
        return g.contiguous(memory_format=torch.channels_last) if ctx.cl else g


class _Frames:
    """T consecutive frames per batch element as one channels-last [b * T, C, H, W] map (the CHM's aligned
    k / v), passed to TrainGraph._hist_cat in place of a [b, heads, T ch, HW] cache view."""

    def __init__(self, x, t):
        self.x, self.t = x, t


def positional_encoding_2d(c: int, h: int, w: int) -> torch.Tensor:
    """Sinusoidal 2-D encoding of the t0 StateAlignBlock (turtle_arch.py:412-439): channels
    [0, c/2) encode the column, [c/2, c) the row, sin on even and cos on odd channels, frequencies
    10000^(-2i / (c/2))."""
    if c % 4:
        raise ValueError(f"Cannot use sin/cos positional encoding with odd dimension (got dim={c})")
    half = c // 2
    freq = torch.exp(torch.arange(0.0, half, 2) * -(math.log(10000.0) / half))      # [half / 2]
    aw = torch.arange(0.0, w)[:, None] * freq                                       # [w, half / 2]
    ah = torch.arange(0.0, h)[:, None] * freq
    pe = torch.empty(c, h, w)
    pe[0:half:2] = torch.sin(aw).t()[:, None, :].expand(-1, h, -1)
    pe[1:half:2] = torch.cos(aw).t()[:, None, :].expand(-1, h, -1)
    pe[half::2] = torch.sin(ah).t()[:, :, None].expand(-1, -1, w)
    pe[half + 1::2] = torch.cos(ah).t()[:, :, None].expand(-1, -1, w)
    return pe


class TrainGraph:
    """The differentiable Turtle_t1 / TurtleSuper_t1 / t0 forward (turtle_t1_arch.py:932-1139,
    turtlesuper_t1_arch.py:1049-1071, turtle_arch.py:459-533) over a ``TurtleParams`` tree.

    Mixed into ``TurtleTrain`` and into the drop-in inference module (``model.TurtleHIP``), which
    routes its forward here whenever autograd is recording and a parameter requires grad, so the
    module ``make_model(opt)`` returns trains under the reference's own loop
    (video_restoration_model.py:78-107). The op set (``graph_ops``) is ``train_ops.HipOps``: the HIP
    kernels, forward and backward; tests inject ATen ops to run the graph on CPU."""

    graph_ops = None            # op-set class; None -> train_ops.HipOps
    sr = False

    def _ops(self):
        ops = self.graph_ops
        if ops is None:
            from .train_ops import HipOps
            ops = HipOps
        return ops

    # ---- blocks (turtle_t1_arch.py:159-811) ------------------------------------------------------
    def _ln(self, m, x):
        return self._ops().layer_norm(x, m.body.weight, getattr(m.body, "bias", None), self.arch.ln_type == "BiasFree")

    def _dw(self, m, x):
        return self._ops().dwconv3x3(x, m.weight, m.bias)

    def _dense(self, x, w, b=None, stride=1, padding=1, groups=1):
        """Dense / window convolutions through F.conv2d - reached by the CPU (ATen) op set only: on the GPU
        the stem / ending, Down / Upsample and SAB window convolutions run on the HIP op set's kernels. A
        channels-last op set gets a standard-layout copy in and channels-last out."""
        cl = getattr(self._ops(), "channels_last", False)
        y = F.conv2d(_ToNCHW.apply(x) if cl else x.contiguous(), w, b, stride, padding, 1, groups)
        return y.contiguous(memory_format=torch.channels_last) if cl else y

    def _conv3(self, x, w):
        """Down / Upsample 3x3 convolution (bias-free, turtle_t1_arch.py:136-154): the op set's implicit-GEMM
        kernel when it has one and the widths allow it, else F.conv2d."""
        ops = self._ops()
        if hasattr(ops, "conv3x3") and w.shape[0] % 8 == 0 and w.shape[1] % 8 == 0:
            return ops.conv3x3(x, w)
        return self._dense(x, w)

    def _conv3_any(self, x, w, b):
        """The stem / ending 3x3 convolutions (input_projection 975-978: 3 (6) -> dim, ending 1035-1041:
        dim -> 3) on the op set's implicit-GEMM kernel with the channel counts zero-padded to multiples of
        8 (a padded input copy of the image, zero weight rows / columns sliced off again), else F.conv2d."""
        ops = self._ops()
        if not hasattr(ops, "conv3x3"):
            return self._dense(x, w, b)
        n, ci = w.shape[0], w.shape[1]
        n8, c8 = -(-n // 8) * 8, -(-ci // 8) * 8
        if c8 != ci:
            xp = torch.empty((x.shape[0], c8, x.shape[2], x.shape[3]), dtype=x.dtype, device=x.device,
                             memory_format=torch.channels_last).zero_()
            xp[:, :ci] = x
            x = xp
        wp = F.pad(w, (0, 0, 0, 0, 0, c8 - ci, 0, n8 - n)) if (c8 != ci or n8 != n) else w
        bp = None if b is None else (F.pad(b, (0, n8 - n)) if n8 != n else b)
        y = ops.conv3x3(x, wp, bp)
        return y[:, :n] if n8 != n else y

    def _c1(self, m, x, res=None):                  # nn.Conv2d(K, N, 1): the op set's GEMM when it has one
        ops = self._ops()
        if hasattr(ops, "conv1x1"):
            return ops.conv1x1(x, m.weight, m.bias, **_res(res))
        return _plus(res, _conv1(m, x))

    def _c1_scaled(self, m, x, scale, res=None):
        """nn.Conv2d(K, N, 1)(x) * scale (scale [1, N, 1, 1]: FeedForward's gamma, ReducedAttn's
        beta) with the scale folded into the weights and bias - W' = diag(scale) W, b' = scale b, tiny
        ops autograd differentiates - so the full-size multiply and its two backward passes (the
        input gradient and gamma's reduction over every pixel) do not run on the op set's GEMM."""
        ops = self._ops()
        if not hasattr(ops, "conv1x1"):
            return _plus(res, _conv1(m, x) * scale)
        sv = scale.reshape(-1)
        w = m.weight.reshape(m.weight.shape[0], m.weight.shape[1]) * sv[:, None]
        b = None if m.bias is None else m.bias * sv
        return ops.conv1x1(x, w, b, **_res(res))

    # ``res`` (every branch): the block's residual stream, returned as res + branch(x) - on op sets
    # with fused residuals the add is the last GEMM's epilogue (turtle_t1_arch.py:808-809)
    def _gffw(self, m, x, res=None):                # GatedFeedForward 159-178
        return self._c1(m.project_out, self._ops().gelu_gate(self._dw(m.dwconv, self._c1(m.project_in, x))), res)

    def _gelu(self, x):
        ops = self._ops()
        return ops.gelu(x) if hasattr(ops, "gelu") else F.gelu(x)

    def _ffw(self, m, x, res=None):                 # FeedForward 181-210
        return self._c1_scaled(m.conv5, self._gelu(self._c1(m.conv4, x)), m.gamma, res)

    def _reduced(self, m, x, res=None):             # ReducedAttn 704-742
        return self._c1_scaled(m.conv3, self._gelu(self._dw(m.conv2, self._c1(m.conv1, x))), m.beta, res)

    def _window(self, x, conv, ws, g):
        """SAB window convolution (k2_dwconv / q2_dwconv: ws x ws, stride ws, padding 1, groups = channels;
        turtle_t1_arch.py:306-308) -> tokens [b, 1, 1, n, g]: on the op set's kernel when it has one
        (channels-last output, whose [b, n, g] view is free), else F.conv2d."""
        ops = self._ops()
        b = x.shape[0]
        if hasattr(ops, "window_conv"):
            y = ops.window_conv(x, conv.weight, conv.bias, ws)
            th, tw = y.shape[2], y.shape[3]
            return y.permute(0, 2, 3, 1).reshape(b, 1, 1, th * tw, g), th, tw
        y = self._dense(x, conv.weight, conv.bias, ws, 1, g)
        th, tw = y.shape[2], y.shape[3]
        return y.reshape(b, g, th * tw).transpose(1, 2).reshape(b, 1, 1, th * tw, g), th, tw

    @staticmethod
    def _heads(t, heads):
        b, c, h, w = t.shape
        return t.reshape(b, heads, c // heads, h * w)

    def _chan(self, m, x, heads, kc=None, vc=None, ntc=None, res=None):
        """ChannelAttention 666-702; with caches / ntc: FrameHistoryRouter 218-286."""
        b, c, h, w = x.shape
        qkv = self._dw(m.qkv_dwconv, self._c1(m.qkv, x))
        ops = self._ops()
        if ntc is None and kc is None and vc is None and hasattr(ops, "norm_gram"):
            # on the op set's kernels: the Gram of the L2-normalised q, k (690-697) in one op over
            # the channel-adjacent [q | k] rows, softmax, then project_out . blockdiag(A) as one
            # per-image weight set applied to v (A v followed by project_out, 697-702)
            # the [q | k] and v slices' input gradients land in one buffer (GradSink): no concatenation
            # in the split's backward
            sink = ops.grad_sink(qkv) if getattr(ops, "grad_sink", None) and qkv.is_contiguous(
                memory_format=torch.channels_last) and not qkv.is_contiguous() else None
            qk, v = _split(qkv, 2 * c, c, sink=sink)
            ch = c // heads
            kw = lambda off: {} if sink is None else {"sink": (sink, off)}
            Gn = ops.norm_gram(qk, heads, **kw(0))
            wp = m.project_out.weight.reshape(c, heads, ch)
            if hasattr(ops, "attn_weff"):           # softmax + W_eff as one op with its own backward
                weff = ops.attn_weff(Gn, m.temperature, wp, _act_dt(v))
            else:
                a = torch.softmax(Gn * m.temperature, dim=-1)
                weff = torch.einsum("ohi,bhij->bohj", wp, a).reshape(b, c, c)
            return ops.conv1x1(v, weff, m.project_out.bias, **kw(2 * c), **_res(res)), None, None
        if ntc is None and kc is None and vc is None and hasattr(ops, "gram"):
            # on the op set's kernels: Gram of the raw q, k over HW (per head) divided by the L2
            # norms (== normalising first, 690-693), softmax, then project_out . blockdiag(A) as
            # one per-image weight set applied to v (A v followed by project_out, 697-702)
            q, k, v = _split(qkv, c, c, c)
            ch = c // heads
            G = ops.gram(q, k, heads)                                          # [b, heads, ch, ch]
            nq = q.float().square().sum((2, 3)).sqrt().clamp_min(L2_EPS).view(b, heads, ch, 1)
            nk = k.float().square().sum((2, 3)).sqrt().clamp_min(L2_EPS).view(b, heads, 1, ch)
            a = torch.softmax(G / (nq * nk) * m.temperature, dim=-1)
            wp = m.project_out.weight.reshape(c, heads, ch)
            weff = torch.einsum("ohi,bhij->bohj", wp, a).reshape(b, c, c)
            return ops.conv1x1(v, weff, m.project_out.bias, **_res(res)), None, None
        if hasattr(ops, "cross_gram"):
            return self._chan_hist(m, qkv, heads, kc, vc, ntc, res)
        q, k, v = _split(qkv, c, c, c)
        q, k, v = _l2n(self._heads(q, heads), -1), _l2n(self._heads(k, heads), -1), self._heads(v, heads)
        if kc is not None and vc is not None:
            k = torch.cat([kc.to(k.dtype), k], dim=2)
            v = torch.cat([vc.to(v.dtype), v], dim=2)
        a = torch.softmax(q @ k.transpose(-2, -1) * m.temperature, dim=-1)
        out = self._c1(m.project_out, (a @ v).reshape(b, c, h, w), res)
        if ntc is None:
            return out, None, None
        keep = int(ntc * c / heads)
        return out, k[:, :, -keep:, :], v[:, :, -keep:, :]

    @staticmethod
    def _hist_cat(cache, cur, heads):
        """[cache ; cur] per head as a channels-last [b, heads * (T+1) * ch, h, w] tensor, head-major
        (channel h (T+1) ch + t ch + i: a head's rows are its cached frames, then the current one, as
        torch.cat(dim=2) of the [b, heads, rows, HW] views, turtle_t1_arch.py:238-240). ``cache``: None,
        a [b, heads, T ch, HW] view (the reference layout, or a slice of an earlier result of this), or
        a ``_Frames`` (CHM: T per-frame channels-last maps of the batch)."""
        b, c, h, w = cur.shape
        ch = c // heads
        if cache is None:
            return cur, 0
        cur6 = cur.permute(0, 2, 3, 1).reshape(b, h, w, heads, 1, ch)
        if isinstance(cache, _Frames):
            t = cache.t
            c6 = cache.x.permute(0, 2, 3, 1).reshape(b, t, h, w, heads, ch).permute(0, 2, 3, 4, 1, 5)
        else:
            t = cache.shape[2] // ch
            c6 = cache.permute(0, 3, 1, 2).reshape(b, h, w, heads, t, ch)
        out = torch.cat([c6.to(cur.dtype), cur6], dim=4)
        return out.reshape(b, h, w, heads * (t + 1) * ch).permute(0, 3, 1, 2), t

    def _chan_hist(self, m, qkv, heads, kc, vc, ntc, res=None):
        """FrameHistoryRouter / the CHM's channel attention over the cached frames (turtle_t1_arch.py:218-286,
        649-660) on the op set's kernels: q, k L2-normalised over HW per channel (norm_cols), the scores
        q_hat [k_cache ; k_hat]^T of all head pairs as one reduction GEMM (cross_gram; each head's block
        taken), softmax, then project_out . blockdiag(A) as one per-image weight set applied to
        [v_cache ; v] - the A v product and project_out in one GEMM, as the inference path does."""
        ops = self._ops()
        c = qkv.shape[1] // 3
        b, _, h, w = qkv.shape
        ch = c // heads
        q, k, v = _split(qkv, c, c, c)
        qn, kn = ops.norm_cols(q), ops.norm_cols(k)
        K, t = self._hist_cat(kc, kn, heads)
        V, _ = self._hist_cat(vc, v, heads)
        L = (t + 1) * ch
        G = ops.cross_gram(qn, K)                                           # [b, c, heads * L]
        Gh = G.view(b, heads, ch, heads, L).diagonal(dim1=1, dim2=3).permute(0, 3, 1, 2)   # [b, heads, ch, L]
        wp = m.project_out.weight.reshape(c, heads, ch)
        if hasattr(ops, "attn_weff"):
            weff = ops.attn_weff(Gh, m.temperature, wp, _act_dt(V))
        else:
            a = torch.softmax(Gh * m.temperature, dim=-1)
            weff = torch.einsum("ohi,bhik->bohk", wp, a).reshape(b, c, heads * L)
        out = ops.conv1x1(V, weff, m.project_out.bias, **_res(res))
        if ntc is None:
            return out, None, None
        keep = int(ntc * c / heads)
        s0 = max(0, L - keep)
        view = lambda T: T.permute(0, 2, 3, 1).reshape(b, h * w, heads, L)[:, :, :, s0:].permute(0, 2, 3, 1)
        return out, view(K), view(V)

    def _ball_mask(self, th, tw, dev, dtype):
        cache = self.__dict__.setdefault("_ball", {})
        key = (th, tw, dev, dtype)
        if key not in cache:
            i = torch.arange(th, device=dev).repeat_interleave(tw)
            j = torch.arange(tw, device=dev).repeat(th)
            cache[key] = (((i[:, None] - i[None, :]).abs() + (j[:, None] - j[None, :]).abs()) <= SAB_RADIUS).to(dtype)
        return cache[key]

    @staticmethod
    def _dilated(t, ws):
        """'b d (p1 h) (p2 w) -> b 1 1 (h w) (p1 p2 d)' (turtle_t1_arch.py:573-574)."""
        b, c, hl, wl = t.shape
        hh, ww = hl // ws, wl // ws
        return t.reshape(b, c, ws, hh, ws, ww).permute(0, 3, 5, 2, 4, 1).reshape(b, 1, 1, hh * ww, ws * ws * c)

    @staticmethod
    def _dilated_t(t, ws):
        """_dilated transposed: [b, 1, ws*ws*c, (h w)] (value tokens as columns)."""
        b, c, hl, wl = t.shape
        hh, ww = hl // ws, wl // ws
        return t.reshape(b, c, ws, hh, ws, ww).permute(0, 2, 4, 1, 3, 5).reshape(b, 1, ws * ws * c, hh * ww)

    @staticmethod
    def _undilated(o, bt, c, hl, wl, ws, cl=False):
        """Inverse of _dilated; ``cl``: the same values as a channels-last [bt, c, hl, wl] tensor (one
        NHWC copy instead of an NCHW one the next GEMM would re-lay out)."""
        hh, ww = hl // ws, wl // ws
        if cl:
            return o.reshape(bt, hh, ww, ws, ws, c).permute(0, 3, 1, 4, 2, 5).reshape(bt, hl, wl, c).permute(0, 3, 1, 2)
        return o.reshape(bt, hh, ww, ws, ws, c).permute(0, 5, 3, 1, 4, 2).reshape(bt, c, hl, wl)

    def _sab(self, m, x, ws, ntc, kc, vc):
        """StateAlignBlock live forward 548-610 (top-5 394-416, L1 ball 448-464, clipped_softmax 115-132)."""
        b, c, hl, wl = x.shape
        qk = self._dw(m.qk_dwconv, self._c1(m.qk, x))
        q, k = _split(qk, c, c)
        v = self._dw(m.v_dwconv, self._c1(m.v, x))
        g = 2 * c
        k, _, _ = self._window(self._c1(m.k2, k), m.k2_dwconv, ws, g)
        q, th, tw = self._window(self._c1(m.q2, q), m.q2_dwconv, ws, g)
        hh, ww = hl // ws, wl // ws
        if th * tw != hh * ww:
            raise RuntimeError(f"SAB q/k token grid {th}x{tw} != v token grid {hh}x{ww} (turtle_t1_arch.py:599)")
        n = th * tw
        q = _l2n(q, -1)
        k = _l2n(k, -1)
        ops = self._ops()
        if _sab_hip_ok(ops, "sab_attention", n, g, ws * ws * c):
            # the values as transposed tokens [b, 1, D, n] (written so by the dilation copy; the cache views
            # handed back are their [b, t, 1, n, D] transposes), scores / top-5 / softmax / A.v on HIP
            vT = self._dilated_t(v, ws)
            K = k.reshape(b, 1, n, g)
            if kc is not None and vc is not None:
                K = torch.cat([kc.reshape(b, -1, n, g).to(K.dtype), K], dim=1)
                vT = torch.cat([vc.reshape(b, -1, n, ws * ws * c).transpose(-1, -2).to(vT.dtype), vT], dim=1)
            t = K.shape[1]
            o = ops.sab_attention(q.reshape(b, n, g), K, vT, m.temperature, tw, SAB_RADIUS)     # [b, t, n, D]
            o = self._undilated(o, b * t, c, hl, wl, ws, getattr(ops, "channels_last", False))
            o = self._c1(m.project_out, o).reshape(b, t, c, hl, wl)
            return o, K[:, -ntc:].unsqueeze(2), vT[:, -ntc:].transpose(-1, -2).unsqueeze(2)
        vt = self._dilated(v, ws)
        if kc is not None and vc is not None:
            k = torch.cat([kc.to(k.dtype), k], dim=1)
            vt = torch.cat([vc.to(vt.dtype), vt], dim=1)
        t = k.shape[1]
        s = (q @ k.transpose(-2, -1)) * m.temperature                   # [b, t, 1, n, n]
        ops = self._ops()
        if _sab_hip_ok(ops, "sab_softmax", n):
            a = ops.sab_softmax(s, tw, SAB_RADIUS)
            o = self._undilated(a @ vt, b * t, c, hl, wl, ws, getattr(ops, "channels_last", False))
            o = self._c1(m.project_out, o).reshape(b, t, c, hl, wl)
            return o, k[:, -ntc:], vt[:, -ntc:]
        top = torch.zeros_like(s).scatter_(-1, torch.topk(s, SAB_TOPK, dim=-1).indices, 1.0)
        # s * top + s * ball as s * (top + ball): the same values bit for bit (factors 0 / 1 / 2 are
        # exact), one full-size pass fewer forward and backward
        s = s * top.add_(self._ball_mask(th, tw, s.device, s.dtype))
        zero = s == 0
        p = torch.softmax(s.masked_fill(zero, float("-inf")), dim=-1).masked_fill(zero, 0.0)
        a = p / p.sum(dim=-1, keepdim=True)
        o = self._undilated(a @ vt, b * t, c, hl, wl, ws, getattr(self._ops(), "channels_last", False))
        o = self._c1(m.project_out, o).reshape(b, t, c, hl, wl)
        return o, k[:, -ntc:], vt[:, -ntc:]

    def _sab_t0(self, m, x, ws, ntc, kc, vc):
        """StateAlignBlock of the t0 network (turtle_arch.py:459-533): the attention it computes is
        discarded (`out = v`, 521-523), so the output is project_out of every frame's v; the caches
        are the last ntc frames of the dilated, L2-normalised k (positional encoding on the qk input,
        412-439) and of v."""
        b, c, hl, wl = x.shape
        pos = positional_encoding_2d(c, hl, wl).to(device=x.device, dtype=x.dtype)
        qk = self._dw(m.qk_dwconv, self._c1(m.qk, x + pos))
        k = qk[:, c:]
        v = self._dw(m.v_dwconv, self._c1(m.v, x))
        if (hl // ws) * (wl // ws) < SAB_TOPK:
            raise RuntimeError("selected index k out of range")
        kt = _l2n(self._dilated(k, ws), -1)
        vt = self._dilated(v, ws)
        if kc is not None and vc is not None:
            kt = torch.cat([kc.to(kt.dtype), kt], dim=1)
            vt = torch.cat([vc.to(vt.dtype), vt], dim=1)
        t = vt.shape[1]
        o = self._c1(m.project_out, self._undilated(vt, b * t, c, hl, wl, ws)).reshape(b, t, c, hl, wl)
        return o, kt[:, -ntc:], vt[:, -ntc:]

    def _chm(self, m, x, heads, ws, ntc, kc, vc, res=None):
        """CausalHistoryModel 612-662."""
        b, c, h, w = x.shape
        sab = self._sab_t0 if self.arch.t0 else self._sab
        xs, k_keep, v_keep = sab(m.spatial_aligner, x, ws, ntc, kc, vc)
        t = xs.shape[1]
        kv = self._dw(m.kv_dwconv, self._c1(m.kv, xs.reshape(b * t, c, h, w)))
        kh, vh = _split(kv, c, c)
        ops = self._ops()
        if hasattr(ops, "cross_gram"):
            # the aligned frames' k, v as per-frame channels-last maps: the history concatenation
            # (_hist_cat) reads them in place; k L2-normalised per frame and channel over HW (649-651)
            out, _, _ = self._chan(m.ChanAttn, x, heads, _Frames(ops.norm_cols(kh), t), _Frames(vh, t), ntc=1, res=res)
            return out, k_keep, v_keep
        ch = c // heads
        kh = kh.reshape(b, t, heads, ch, h * w).transpose(1, 2).reshape(b, heads, t * ch, h * w)
        vh = vh.reshape(b, t, heads, ch, h * w).transpose(1, 2).reshape(b, heads, t * ch, h * w)
        out, _, _ = self._chan(m.ChanAttn, x, heads, _l2n(kh, -1), vh, ntc=1, res=res)
        return out, k_keep, v_keep

    def _ln_res(self, m, x):
        """(LayerNorm(x), r): r is x for the residual add - on op sets with fused residuals an alias
        whose gradient the LayerNorm backward sums into its own (no separate gradient add), else None
        (the branch result is added as written)."""
        ops = self._ops()
        if getattr(ops, "fused_residual", False):
            return ops.layer_norm(x, m.body.weight, getattr(m.body, "bias", None), self.arch.ln_type == "BiasFree",
                                  residual=True)
        return self._ln(m, x), None

    def _block(self, spec, m, x, kc=None, vc=None):
        """TurtleAttnBlock 804-811: x = x + attn(norm1(x)); x = x + ffn(norm2(x))."""
        k_out = v_out = None
        if spec.attn != "NoAttn":
            y, r = self._ln_res(m.norm1, x)
            if spec.attn == "ReducedAttn":
                a = self._reduced(m.attn, y, r)
            elif spec.attn == "Channel":
                a, _, _ = self._chan(m.attn, y, spec.heads, res=r)
            elif spec.attn == "FHR":
                a, k_out, v_out = self._chan(m.attn, y, spec.heads, kc, vc, ntc=spec.ntc, res=r)
            else:
                a, k_out, v_out = self._chm(m.attn, y, spec.heads, spec.ws, spec.ntc, kc, vc, res=r)
            x = a if r is not None else x + a
        y, r = self._ln_res(m.norm2, x)
        f = self._gffw(m.ffn, y, r) if spec.ffn == "GFFW" else self._ffw(m.ffn, y, r)
        x = f if r is not None else x + f
        return x, k_out, v_out

    def _level(self, name, x, kc=None, vc=None):    # LevelBlock 856-865
        specs, mods = self.arch.levels[name].blocks, getattr(self, name).transformer_blocks
        for s, m in zip(specs[:-1], mods[:-1]):
            x, _, _ = self._block(s, m, x)
        return self._block(specs[-1], mods[-1], x, kc, vc)

    def _latent(self, x, k1, v1, k2, v2):          # LatentCacheBlock 919-928
        specs, mods = self.arch.levels["latent"].blocks, self.latent.transformer_blocks
        x, k1o, v1o = self._block(specs[0], mods[0], x, k1, v1)
        for s, m in zip(specs[1:-1], mods[1:-1]):
            x, _, _ = self._block(s, m, x)
        x, k2o, v2o = self._block(specs[-1], mods[-1], x, k2, v2)
        return x, k1o, v1o, k2o, v2o

    def graph_forward(self, inp_img_: torch.Tensor, k_cached: Optional[List] = None, v_cached: Optional[List] = None):
        """Turtle_t1.forward 1045-1132 (TurtleSuper_t1: bilinear x4 first, turtlesuper_t1_arch.py:
        1049-1071): [B, 2, C, H, W] -> (out [B, C, H, W] (x4 for SR), k_list[8], v_list[8])."""
        b, _, c, h, w = inp_img_.shape
        if k_cached is None:
            k_cached, v_cached = [None] * 8, [None] * 8
        if self.sr:
            if self.arch.use_both:      # turtlesuper_t1_arch.py:1059-1065 never defines `current` there
                raise ValueError("TurtleSuper_t1 with use_both_input=True is not runnable in the reference")
            h, w = 4 * h, 4 * w
            src = F.interpolate(inp_img_[:, 1], scale_factor=4, mode="bilinear", align_corners=False)
            ph, pw = (32 - h % 32) % 32, (32 - w % 32) % 32
            img = F.pad(src, (0, pw, 0, ph)) if ph or pw else src
            current = img[:, -c:]
        else:
            ph, pw = (32 - h % 32) % 32, (32 - w % 32) % 32
            x5 = F.pad(inp_img_, (0, pw, 0, ph)) if ph or pw else inp_img_
            current = x5[:, 1]
            img = torch.cat([x5[:, 0], x5[:, 1]], dim=1) if self.arch.use_both else current
        ip = self.input_projection
        e1 = self._conv3_any(img.float(), ip.weight, ip.bias)
        ks, vs = [], []
        e1, k, v = self._level("encoder_level1", e1, k_cached[0], v_cached[0]); ks.append(k); vs.append(v)
        # Downsample 136-144 / Upsample 146-154. On the channels-last op set the shuffled map is made
        # channels-last once here (pixel_(un)shuffle returns NCHW on ROCm): otherwise the next level's
        # residual stream stays NCHW and every LayerNorm / GEMM of the level re-lays its input out
        cl = (lambda t: t.contiguous(memory_format=torch.channels_last)) if getattr(self._ops(), "channels_last", False) \
            else (lambda t: t)
        down = lambda m, t: cl(F.pixel_unshuffle(self._conv3(t, m.body[0].weight), 2))
        up = lambda m, t: cl(F.pixel_shuffle(self._conv3(t, m.body[0].weight), 2))
        e2, k, v = self._level("encoder_level2", down(self.down1_2, e1), k_cached[1], v_cached[1]); ks.append(k); vs.append(v)
        e3, k, v = self._level("encoder_level3", down(self.down2_3, e2), k_cached[2], v_cached[2]); ks.append(k); vs.append(v)
        lat, k1, v1, k2, v2 = self._latent(down(self.down3_4, e3), k_cached[3], v_cached[3], k_cached[4], v_cached[4])
        ks += [k1, k2]; vs += [v1, v2]
        d3 = self._c1(self.reduce_chan_level3, torch.cat([up(self.up4_3, lat), e3], 1))
        d3, k, v = self._level("decoder_level3", d3, k_cached[5], v_cached[5]); ks.append(k); vs.append(v)
        d2 = self._c1(self.reduce_chan_level2, torch.cat([up(self.up3_2, d3), e2], 1))
        d2, k, v = self._level("decoder_level2", d2, k_cached[6], v_cached[6]); ks.append(k); vs.append(v)
        d1 = self._c1(self.reduce_chan_level1, torch.cat([up(self.up2_1, d2), e1], 1))
        d1, k, v = self._level("decoder_level1", d1, k_cached[7], v_cached[7]); ks.append(k); vs.append(v)
        r, _, _ = self._level("refinement", d1)
        out = self._conv3_any(r, self.ending.weight, self.ending.bias) + current
        return out[:, :, :h, :w], ks, vs


class TurtleTrain(TrainGraph, TurtleParams):
    """Differentiable Turtle_t1 (turtle_t1_arch.py:932-1139) for the training step; ``ops`` supplies
    layer_norm, dwconv3x3 and gelu_gate (``train_ops.HipOps`` on the GPU)."""

    def __init__(self, opt: dict, ops=None, sr: bool = False):
        TurtleParams.__init__(self, opt)
        self.sr = sr
        if ops is not None:
            self.graph_ops = ops

    def forward(self, inp_img_: torch.Tensor, k_cached: Optional[List] = None, v_cached: Optional[List] = None):
        return self.graph_forward(inp_img_, k_cached, v_cached)


class Trainer:
    """One optimisation step per call, as VideoRestorationModel.optimize_parameters (78-108).

    ``amp``: "bf16" (MI355X default: bf16 autocast, no loss scaling), "fp16" (the reference's
    autocast + GradScaler) or None (fp32). With an initialised process group the network is wrapped
    in DistributedDataParallel (RCCL on ROCm) with ``bucket_mb`` gradient buckets."""

    def __init__(self, net: TurtleTrain, lr: float = 4e-4, betas=(0.9, 0.99), weight_decay: float = 0.0,
                 amp: Optional[str] = "bf16", bucket_mb: int = 64, accumulate_grads: bool = True):
        self.net = net
        self.world = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
        dev = next(net.parameters()).device
        self.device = dev
        if self.world > 1:
            kw = dict(device_ids=[dev.index]) if dev.type == "cuda" else {}
            self.model = torch.nn.parallel.DistributedDataParallel(
                net, find_unused_parameters=False, bucket_cap_mb=bucket_mb, gradient_as_bucket_view=True, **kw)
        else:
            self.model = net
        self.opt = torch.optim.AdamW([{"params": [p for p in net.parameters() if p.requires_grad]}], lr=lr, betas=betas,
                                     weight_decay=weight_decay)
        self.amp = amp
        self.scaler = torch.amp.GradScaler("cuda", enabled=(amp == "fp16" and dev.type == "cuda"))
        # the op set's in-place parameter-gradient accumulation (train_ops.ParamGradAccumulator):
        # one fp32 arena per step instead of per-use gradients added by autograd
        make_acc = getattr(net._ops(), "param_grad_accumulator", None) if accumulate_grads else None
        self.acc = make_acc(list(net.parameters())) if make_acc is not None else None

    def _autocast(self):
        if self.amp is None or self.device.type != "cuda":
            return torch.autocast(device_type=self.device.type, enabled=False)
        return torch.autocast(device_type="cuda", dtype=torch.bfloat16 if self.amp == "bf16" else torch.float16)

    def loss(self, lq: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
        """Frame-averaged L1 over the causal loop (video_restoration_model.py:84-98); caches are
        carried un-detached (BPTT through the history)."""
        T = lq.shape[1]
        kc = vc = None
        total = 0.0
        with self._autocast():
            for j in range(T):
                inp = torch.stack([lq[:, j if j == 0 else j - 1], lq[:, j]], dim=1)
                out, kc, vc = self.model(inp, kc, vc)
                total = total + F.l1_loss(out.float(), gt[:, j].float())
        return total / T

    def backward(self, lq: torch.Tensor, gt: torch.Tensor) -> torch.Tensor:
        """Forward and backward of one iteration (video_restoration_model.py:84-102): the parameter
        gradients (scaled under fp16) land in ``.grad``; returns the detached pixel loss. With the
        op set's accumulator every weight gradient is summed in place over the clip's frames."""
        self.opt.zero_grad(set_to_none=True)
        if self.acc is not None:
            with self.acc.step():
                l_pix = self.loss(lq, gt)
                l_total = l_pix + self.acc.zero_term(list(self.net.parameters()))
                self.scaler.scale(l_total).backward()
        else:
            l_pix = self.loss(lq, gt)
            l_total = l_pix + 0 * sum(p.sum() for p in self.net.parameters())
            self.scaler.scale(l_total).backward()
        return l_pix.detach()

    def train_step(self, lq: torch.Tensor, gt: torch.Tensor) -> float:
        """One iteration; returns the loss averaged over ranks (valid on rank 0, like
        reduce_loss_dict)."""
        l_pix = self.backward(lq, gt)
        self.scaler.unscale_(self.opt)
        self.scaler.step(self.opt)
        self.scaler.update()
        red = l_pix.clone()
        if self.world > 1:                           # base_model.py:340-365: reduce to rank 0, / world
            dist.reduce(red, dst=0)
            if dist.get_rank() == 0:
                red /= self.world
        return float(red)
