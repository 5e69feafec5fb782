"""CPU oracle: a functional fp32 restatement of the Turtle_t1 / TurtleSuper_t1 forward.

TEST INFRASTRUCTURE ONLY. Nothing in the product path (``turtlevsr_amd``, ``basicsr``) imports
this module; only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg use it, as the checker / the CPU baseline.

It restates the reference algorithm from its semantics (not its code): plain torch CPU ops on a
``{name: tensor}`` state dict, following the live definitions of
``/root/reference/basicsr/models/archs/turtle_t1_arch.py`` (cited per function below) and the SR
front-end of ``turtlesuper_t1_arch.py:976-977,1049-1071``.

Parity pin: it is checked against golden vectors produced by the reference itself in the
build container (``tests/golden/gen_golden.py`` loads the reference arch by file path). See
``tests/test_oracle_golden.py``.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

Tensor = torch.Tensor
SD = Dict[str, Tensor]

LN_EPS = 1e-5      # turtle_t1_arch.py:81,99 (inside the sqrt)
L2_EPS = 1e-12     # F.normalize default, used at 265-266, 577-578, 657, 690-691
SAB_TOPK = 5       # turtle_t1_arch.py:588
SAB_RADIUS = 4     # turtle_t1_arch.py:590 (L1 distance on the token grid)
PAD_MULT = 32      # turtle_t1_arch.py:1043 padder_size = 2**3 * 4

# A.v of the StateAlignBlock as a sparse product: the clipped-softmax rows have at most top-5 + the
# 41-key L1 ball non-zeros, so a @ v (turtle_t1_arch.py:600) is the same sum over those keys. Off by
# default (the CPU baseline times the reference's dense product); the 1080p parity test turns it on
# so that one steady-state 1920x1088 oracle frame (N = 8160 tokens) fits a test's time budget.
SAB_SPARSE_AV = False


# ----------------------------------------------------------------------------------------------
# Architecture description (make_model, turtle_t1_arch.py:10-53; Turtle_t1.__init__ 932-1043)
# ----------------------------------------------------------------------------------------------
@dataclass
class Block:
    prefix: str            # e.g. "decoder_level1.transformer_blocks.1"
    dim: int
    attn: str              # ReducedAttn | Channel | FHR | CHM | NoAttn
    ffn: str               # FFW | GFFW
    heads: int
    ntc: int               # num_frames_tocache
    ws: int                # SAB window size = 2 * Scale_patchsize
    t0: bool = False       # "Turtle" (turtle_arch.py) StateAlignBlock instead of Turtle_t1's


@dataclass
class Level:
    name: str
    blocks: List[Block] = field(default_factory=list)


def arch_from_opt(opt: dict) -> dict:
    """Resolve an option dict into the level/block list (defaults as make_model)."""
    dim = opt["dim"]
    heads = opt.get("num_heads", [1, 1, 1, 1])
    ntc = opt.get("num_frames_tocache", 1)
    ffe = opt.get("ffn_expansion_factor", 1)

    def level(name, d, n, t1, t2, ffw, h, nt, scale):
        lv = Level(name)
        for i in range(n):
            a = t2 if i == n - 1 else t1
            lv.blocks.append(Block(f"{name}.transformer_blocks.{i}", d, a, ffw, h, nt, 2 * scale))
        return lv

    def latent(name, d, n, t1, t2, t3, ffw, h, nt):
        if n < 2:
            raise ValueError("LatentCacheBlock needs at least 2 blocks")  # 899-901
        lv = Level(name)
        for i in range(n):
            a = t1 if i == 0 else (t3 if i == n - 1 else t2)
            lv.blocks.append(Block(f"{name}.transformer_blocks.{i}", d, a, ffw, h, nt, 2))
        return lv

    eb, db = opt["Enc_blocks"], opt["Dec_blocks"]
    o = opt
    levels = {
        "encoder_level1": level("encoder_level1", dim, eb[0], o["encoder1_attn_type1"], o["encoder1_attn_type2"], o["encoder1_ffw_type"], heads[0], ntc, 1),
        "encoder_level2": level("encoder_level2", dim * 2, eb[1], o["encoder2_attn_type1"], o["encoder2_attn_type2"], o["encoder2_ffw_type"], heads[1], ntc, 1),
        "encoder_level3": level("encoder_level3", dim * 4, eb[2], o["encoder3_attn_type1"], o["encoder3_attn_type2"], o["encoder3_ffw_type"], heads[2], ntc, 1),
        "latent": latent("latent", dim * 8, o["Middle_blocks"], o["latent_attn_type1"], o["latent_attn_type2"], o["latent_attn_type3"], o["latent_ffw_type"], heads[3], ntc),
        # decoder_level3/2/1 use the decoder1/2/3 keys (1009-1027); Scale_patchsize 2/4/8;
        # decoder_level1 forces num_frames_tocache=2 (1027)
        "decoder_level3": level("decoder_level3", dim * 4, db[0], o["decoder1_attn_type1"], o["decoder1_attn_type2"], o["decoder1_ffw_type"], heads[2], ntc, 2),
        "decoder_level2": level("decoder_level2", dim * 2, db[1], o["decoder2_attn_type1"], o["decoder2_attn_type2"], o["decoder2_ffw_type"], heads[1], ntc, 4),
        "decoder_level1": level("decoder_level1", dim, db[2], o["decoder3_attn_type1"], o["decoder3_attn_type2"], o["decoder3_ffw_type"], heads[0], 2, 8),
        "refinement": level("refinement", dim, opt.get("num_refinement_blocks", 1), o["refinement_attn_type1"], o["refinement_attn_type2"], o["refinement_ffw_type"], heads[0], ntc, 1),
    }
    known = {"ReducedAttn", "Channel", "FHR", "CHM", "NoAttn"}
    t0 = is_t0(opt)
    for lv in levels.values():
        for b in lv.blocks:
            b.t0 = t0
            if b.attn not in known:
                raise ValueError(f"attention type {b.attn!r} not defined")
            if b.ffn not in ("FFW", "GFFW"):
                raise ValueError(f"FFW type {b.ffn!r} not defined")
    return dict(levels=levels, dim=dim, ffe=ffe, use_both=bool(opt["use_both_input"]),
                ln_type=opt.get("LayerNorm_type", "WithBias"), ntc=ntc, t0=t0)


def is_t0(opt: dict) -> bool:
    """The option file's `model` selects the arch module (video_restoration_model.py:18-21):
    Turtle_arch -> the t0 network (turtle_arch.py), otherwise Turtle_t1 / TurtleSuper_t1."""
    return str(opt.get("model", "")).lower() in ("turtle_arch", "turtle")


# ----------------------------------------------------------------------------------------------
# Primitive ops
# ----------------------------------------------------------------------------------------------
def _conv(sd: SD, name: str, x: Tensor, stride=1, padding=0, groups=1) -> Tensor:
    return F.conv2d(x, sd[name + ".weight"], sd.get(name + ".bias"), stride, padding, 1, groups)


def _dw(sd: SD, name: str, x: Tensor) -> Tensor:
    """Depthwise 3x3, pad 1 (e.g. qkv_dwconv 237, conv2 716-722, dwconv 167-169)."""
    return _conv(sd, name, x, 1, 1, x.shape[1])


def layer_norm(sd: SD, name: str, x: Tensor, ln_type: str) -> Tensor:
    """Per-pixel LayerNorm over channels, biased variance, eps inside sqrt (67-112)."""
    mu = x.mean(dim=1, keepdim=True)
    var = ((x - mu) ** 2).mean(dim=1, keepdim=True)
    w = sd[name + ".body.weight"].view(1, -1, 1, 1)
    if ln_type == "BiasFree":
        return x / torch.sqrt(var + LN_EPS) * w
    return (x - mu) / torch.sqrt(var + LN_EPS) * w + sd[name + ".body.bias"].view(1, -1, 1, 1)


def l2n(x: Tensor, dim: int) -> Tensor:
    return x / x.norm(dim=dim, keepdim=True).clamp_min(L2_EPS)


def gated_ffn(sd: SD, p: str, x: Tensor) -> Tensor:
    """GatedFeedForward 159-178: project_in -> dw3x3 -> gelu(x1)*x2 -> project_out."""
    y = _dw(sd, p + ".dwconv", _conv(sd, p + ".project_in", x))
    h = y.shape[1] // 2
    return _conv(sd, p + ".project_out", F.gelu(y[:, :h]) * y[:, h:])


def feed_forward(sd: SD, p: str, x: Tensor) -> Tensor:
    """FeedForward 181-210: conv4 -> gelu -> conv5, times gamma."""
    y = _conv(sd, p + ".conv5", F.gelu(_conv(sd, p + ".conv4", x)))
    return y * sd[p + ".gamma"]


def reduced_attn(sd: SD, p: str, x: Tensor) -> Tensor:
    """ReducedAttn 704-742: conv1 -> dw conv2 (+bias) -> gelu -> conv3, times beta."""
    y = _conv(sd, p + ".conv3", F.gelu(_dw(sd, p + ".conv2", _conv(sd, p + ".conv1", x))))
    return y * sd[p + ".beta"]


def _heads(t: Tensor, heads: int) -> Tensor:
    b, c, h, w = t.shape
    return t.reshape(b, heads, c // heads, h * w)


def channel_attention(sd: SD, p: str, x: Tensor, heads: int) -> Tensor:
    """ChannelAttention 666-702 (transposed / MDTA attention over channels)."""
    b, c, h, w = x.shape
    q, k, v = _dw(sd, p + ".qkv_dwconv", _conv(sd, p + ".qkv", x)).chunk(3, dim=1)
    q, k, v = l2n(_heads(q, heads), -1), l2n(_heads(k, heads), -1), _heads(v, heads)
    a = torch.softmax(q @ k.transpose(-2, -1) * sd[p + ".temperature"], dim=-1)
    return _conv(sd, p + ".project_out", (a @ v).reshape(b, c, h, w))


def frame_history_router(sd: SD, p: str, x: Tensor, heads: int, ntc: int,
                         k_cached: Optional[Tensor], v_cached: Optional[Tensor]):
    """FrameHistoryRouter 218-286: channel attention whose keys/values prepend cached rows.

    Returns (out, k_keep, v_keep); the kept rows are the last ``ntc * c / heads`` rows of the
    concatenated (normalised) k and (raw) v.
    """
    b, c, h, w = x.shape
    q, k, v = _dw(sd, p + ".qkv_dwconv", _conv(sd, p + ".qkv", x)).chunk(3, dim=1)
    q, k, v = l2n(_heads(q, heads), -1), l2n(_heads(k, heads), -1), _heads(v, heads)
    if k_cached is not None and v_cached is not None:
        k = torch.cat([k_cached, k], dim=2)
        v = torch.cat([v_cached, v], dim=2)
    a = torch.softmax(q @ k.transpose(-2, -1) * sd[p + ".temperature"], dim=-1)
    out = _conv(sd, p + ".project_out", (a @ v).reshape(b, c, h, w))
    keep = int(ntc * c / heads)
    return out, k[:, :, -keep:, :], v[:, :, -keep:, :]


def ball_mask(hh: int, ww: int, radius: int = SAB_RADIUS) -> Tensor:
    """Token-grid L1 ball |di|+|dj| <= radius, no wrap (live create_local_attention_mask 448-464)."""
    i = torch.arange(hh).repeat_interleave(ww)
    j = torch.arange(ww).repeat(hh)
    return ((i[:, None] - i[None, :]).abs() + (j[:, None] - j[None, :]).abs()) <= radius


def clipped_softmax(s: Tensor) -> Tensor:
    """clipped_softmax 115-132: softmax over the entries that are not exactly zero, renormalised."""
    zero = s == 0
    p = torch.softmax(s.masked_fill(zero, float("-inf")), dim=-1).masked_fill(zero, 0.0)
    return p / p.sum(dim=-1, keepdim=True)


def state_align(sd: SD, p: str, x: Tensor, ws: int, ntc: int,
                k_cached: Optional[Tensor], v_cached: Optional[Tensor]):
    """StateAlignBlock, live forward 548-610 (+ zero_out_non_top_k 394-416, mask 448-464).

    q/k tokens come from a ws x ws / stride ws / pad 1 depthwise window conv (contiguous windows);
    v tokens are the dilated regroup 'b d (p1 h) (p2 w) -> b 1 1 (h w) (p1 p2 d)'.
    """
    b, c, hl, wl = x.shape
    qk = _dw(sd, p + ".qk_dwconv", _conv(sd, p + ".qk", x))
    q, k = qk[:, :c], qk[:, c:]
    v = _dw(sd, p + ".v_dwconv", _conv(sd, p + ".v", x))
    g = 2 * c
    k = _conv(sd, p + ".k2_dwconv", _conv(sd, p + ".k2", k), ws, 1, g)
    q = _conv(sd, p + ".q2_dwconv", _conv(sd, p + ".q2", q), ws, 1, g)
    th, tw = q.shape[2], q.shape[3]
    n = th * tw
    q = l2n(q.reshape(b, g, n).transpose(1, 2).reshape(b, 1, 1, n, g), -1)
    k = l2n(k.reshape(b, g, n).transpose(1, 2).reshape(b, 1, 1, n, g), -1)
    hh, ww_ = hl // ws, wl // ws
    # v[b, d, p1*hh + i, p2*ww + j] -> token (i, j), feature (p1*ws + p2)*c + d
    vt = v.reshape(b, c, ws, hh, ws, ww_).permute(0, 3, 5, 2, 4, 1).reshape(b, 1, 1, hh * ww_, ws * ws * c)
    if k_cached is not None and v_cached is not None:
        k = torch.cat([k_cached, k], dim=1)
        vt = torch.cat([v_cached, vt], dim=1)
    t = k.shape[1]
    s = (q @ k.transpose(-2, -1)) * sd[p + ".temperature"]           # [b, t, 1, n, n]
    top = torch.zeros_like(s).scatter_(-1, torch.topk(s, SAB_TOPK, dim=-1).indices, 1.0)
    ball = ball_mask(th, tw).to(s.dtype)
    a = clipped_softmax(s * top + s * ball)
    if SAB_SPARSE_AV:
        vb = vt.expand(b, t, 1, n, vt.shape[-1])
        o = torch.stack([torch.sparse.mm(ai.to_sparse(), vi) for ai, vi in
                         zip(a.reshape(-1, n, n), vb.reshape(-1, n, vt.shape[-1]))]).reshape(b, t, 1, n, -1)
    else:
        o = a @ vt                                                    # [b, t, 1, n, ws*ws*c]
    o = o.reshape(b * t, hh, ww_, ws, ws, c).permute(0, 5, 3, 1, 4, 2).reshape(b * t, c, hl, wl)
    o = _conv(sd, p + ".project_out", o).reshape(b, t, c, hl, wl)
    return o, k[:, -ntc:], vt[:, -ntc:]


def positional_encoding_2d(d_model: int, height: int, width: int) -> Tensor:
    """Sinusoidal 2-D encoding of the t0 StateAlignBlock (turtle_arch.py:412-439): the first half
    of the channels encodes the column (sin / cos interleaved), the second half the row."""
    if d_model % 4 != 0:
        raise ValueError(f"Cannot use sin/cos positional encoding with odd dimension (got dim={d_model})")
    pe = torch.zeros(d_model, height, width)
    half = d_model // 2
    div = torch.exp(torch.arange(0.0, half, 2) * -(math.log(10000.0) / half))
    pos_w = torch.arange(0.0, width).unsqueeze(1)
    pos_h = torch.arange(0.0, height).unsqueeze(1)
    pe[0:half:2] = torch.sin(pos_w * div).transpose(0, 1).unsqueeze(1).repeat(1, height, 1)
    pe[1:half:2] = torch.cos(pos_w * div).transpose(0, 1).unsqueeze(1).repeat(1, height, 1)
    pe[half::2] = torch.sin(pos_h * div).transpose(0, 1).unsqueeze(2).repeat(1, 1, width)
    pe[half + 1::2] = torch.cos(pos_h * div).transpose(0, 1).unsqueeze(2).repeat(1, 1, width)
    return pe


def _dilated_tokens(t: Tensor, ws: int) -> Tensor:
    """'b d (p1 h) (p2 w) -> b 1 1 (h w) (p1 p2 d)' (turtle_t1_arch.py:573-574, turtle_arch.py:487-492)."""
    b, c, hl, wl = t.shape
    hh, ww_ = hl // ws, wl // ws
    return t.reshape(b, c, ws, hh, ws, ww_).permute(0, 3, 5, 2, 4, 1).reshape(b, 1, 1, hh * ww_, ws * ws * c)


def state_align_t0(sd: SD, p: str, x: Tensor, ws: int, ntc: int,
                   k_cached: Optional[Tensor], v_cached: Optional[Tensor]):
    """StateAlignBlock of the t0 network, live forward turtle_arch.py:459-533 (the later of the
    class's two `forward` definitions). q/k come from x + a 2-D positional encoding, all of q, k, v
    are dilated token groups (one head), q/k L2-normalised over ws*ws*c. The attention is computed
    and then discarded (`out = v`, 521-523): the output is project_out of every frame's v, the
    caches are the last ntc frames of k and v. The discarded attention still runs top-5 over the
    keys, so fewer than 5 tokens raises like the reference."""
    b, c, hl, wl = x.shape
    pos = positional_encoding_2d(c, hl, wl).to(x.dtype)
    qk = _dw(sd, p + ".qk_dwconv", _conv(sd, p + ".qk", x + pos))
    k = qk[:, c:]
    v = _dw(sd, p + ".v_dwconv", _conv(sd, p + ".v", x))
    hh, ww_ = hl // ws, wl // ws
    if hh * ww_ < SAB_TOPK:
        raise RuntimeError("selected index k out of range")
    kt = l2n(_dilated_tokens(k, ws), -1)
    vt = _dilated_tokens(v, ws)
    if k_cached is not None and v_cached is not None:
        kt = torch.cat([k_cached, kt], dim=1)
        vt = torch.cat([v_cached, vt], dim=1)
    t = vt.shape[1]
    o = vt.reshape(b * t, hh, ww_, ws, ws, c).permute(0, 5, 3, 1, 4, 2).reshape(b * t, c, hl, wl)
    o = _conv(sd, p + ".project_out", o).reshape(b, t, c, hl, wl)
    return o, kt[:, -ntc:], vt[:, -ntc:]


def causal_history(sd: SD, p: str, x: Tensor, heads: int, ws: int, ntc: int,
                   k_cached: Optional[Tensor], v_cached: Optional[Tensor], t0: bool = False):
    """CausalHistoryModel 612-662: SAB -> kv conv on the aligned frames -> FHR(x, k_hist, v_hist)."""
    b, c, h, w = x.shape
    sab = state_align_t0 if t0 else state_align
    xs, k_keep, v_keep = sab(sd, p + ".spatial_aligner", x, ws, ntc, k_cached, v_cached)
    t = xs.shape[1]
    kv = _dw(sd, p + ".kv_dwconv", _conv(sd, p + ".kv", xs.reshape(b * t, c, h, w)))
    kh, vh = kv[:, :c], kv[:, c:]
    # '(b t) (head c) h w -> b head (t c) (h w)'
    kh = kh.reshape(b, t, heads, c // heads, h * w).transpose(1, 2).reshape(b, heads, t * (c // heads), h * w)
    vh = vh.reshape(b, t, heads, c // heads, h * w).transpose(1, 2).reshape(b, heads, t * (c // heads), h * w)
    out, _, _ = frame_history_router(sd, p + ".ChanAttn", x, heads, 1, l2n(kh, -1), vh)
    return out, k_keep, v_keep


def turtle_block(sd: SD, blk: Block, x: Tensor, ln_type: str, ffe: float,
                 k_cached=None, v_cached=None):
    """TurtleAttnBlock 746-811: pre-norm residual attention + pre-norm residual FFN."""
    p = blk.prefix
    kc = vc = None
    if blk.attn != "NoAttn":
        y = layer_norm(sd, p + ".norm1", x, ln_type)
        if blk.attn == "ReducedAttn":
            a = reduced_attn(sd, p + ".attn", y)
        elif blk.attn == "Channel":
            a = channel_attention(sd, p + ".attn", y, blk.heads)
        elif blk.attn == "FHR":
            a, kc, vc = frame_history_router(sd, p + ".attn", y, blk.heads, blk.ntc, k_cached, v_cached)
        else:  # CHM
            a, kc, vc = causal_history(sd, p + ".attn", y, blk.heads, blk.ws, blk.ntc, k_cached, v_cached, blk.t0)
        x = x + a
    y = layer_norm(sd, p + ".norm2", x, ln_type)
    x = x + (gated_ffn(sd, p + ".ffn", y) if blk.ffn == "GFFW" else feed_forward(sd, p + ".ffn", y))
    return x, kc, vc


def _level(sd, arch, name, x, kc=None, vc=None):
    """LevelBlock.forward 856-865: only the last block sees the cache."""
    blocks = arch["levels"][name].blocks
    for blk in blocks[:-1]:
        x, _, _ = turtle_block(sd, blk, x, arch["ln_type"], arch["ffe"])
    return turtle_block(sd, blocks[-1], x, arch["ln_type"], arch["ffe"], kc, vc)


def _latent(sd, arch, x, k1, v1, k2, v2):
    """LatentCacheBlock.forward 919-928: first and last block see caches [3] and [4]."""
    blocks = arch["levels"]["latent"].blocks
    x, k1o, v1o = turtle_block(sd, blocks[0], x, arch["ln_type"], arch["ffe"], k1, v1)
    for blk in blocks[1:-1]:
        x, _, _ = turtle_block(sd, blk, x, arch["ln_type"], arch["ffe"])
    x, k2o, v2o = turtle_block(sd, blocks[-1], x, arch["ln_type"], arch["ffe"], k2, v2)
    return x, k1o, v1o, k2o, v2o


def _down(sd, name, x):   # Downsample 136-144: 3x3 c->c/2, PixelUnshuffle(2)
    return F.pixel_unshuffle(_conv(sd, name + ".body.0", x, 1, 1), 2)


def _up(sd, name, x):     # Upsample 146-154: 3x3 c->2c, PixelShuffle(2)
    return F.pixel_shuffle(_conv(sd, name + ".body.0", x, 1, 1), 2)


def pad_to(x: Tensor, mult: int = PAD_MULT) -> Tensor:
    """check_image_size 1134-1139: zero-pad right/bottom to a multiple of 32."""
    h, w = x.shape[-2:]
    return F.pad(x, (0, (mult - w % mult) % mult, 0, (mult - h % mult) % mult))   # (w, h) order: 1138


@torch.no_grad()
def turtle_forward(sd: SD, opt: dict, inp: Tensor, k_cached=None, v_cached=None, sr: bool = False):
    """Turtle_t1.forward 1045-1132 (``sr=True``: TurtleSuper_t1.forward, turtlesuper 1049-1071).

    ``inp``: [B, 2, C, H, W]. Returns (out [B, C, H', W'], k_list[8], v_list[8]).
    """
    arch = arch_from_opt(opt)
    b, _, c, h, w = inp.shape
    if k_cached is None:
        k_cached, v_cached = [None] * 8, [None] * 8
    if sr:
        if arch["use_both"]:
            # turtlesuper 1059-1065 adds the un-upsampled current frame to a 4x output: the
            # reference itself cannot run this combination.
            raise ValueError("TurtleSuper_t1 with use_both_input=True is not runnable")
        h, w = 4 * h, 4 * w
        img = pad_to(F.interpolate(inp[:, 1], scale_factor=4, mode="bilinear", align_corners=False))
        current = img
    else:
        x5 = pad_to(inp)
        if arch["use_both"]:
            img = torch.cat([x5[:, 0], x5[:, 1]], dim=1)
        else:
            img = x5[:, 1]
        current = x5[:, 1]
    e1 = _conv(sd, "input_projection", img.float(), 1, 1)
    ks, vs = [], []
    e1, k, v = _level(sd, arch, "encoder_level1", e1, k_cached[0], v_cached[0]); ks.append(k); vs.append(v)
    e2, k, v = _level(sd, arch, "encoder_level2", _down(sd, "down1_2", e1), k_cached[1], v_cached[1]); ks.append(k); vs.append(v)
    e3, k, v = _level(sd, arch, "encoder_level3", _down(sd, "down2_3", e2), k_cached[2], v_cached[2]); ks.append(k); vs.append(v)
    lat, k1, v1, k2, v2 = _latent(sd, arch, _down(sd, "down3_4", e3), k_cached[3], v_cached[3], k_cached[4], v_cached[4])
    ks += [k1, k2]; vs += [v1, v2]
    d3 = _conv(sd, "reduce_chan_level3", torch.cat([_up(sd, "up4_3", lat), e3], 1))
    d3, k, v = _level(sd, arch, "decoder_level3", d3, k_cached[5], v_cached[5]); ks.append(k); vs.append(v)
    d2 = _conv(sd, "reduce_chan_level2", torch.cat([_up(sd, "up3_2", d3), e2], 1))
    d2, k, v = _level(sd, arch, "decoder_level2", d2, k_cached[6], v_cached[6]); ks.append(k); vs.append(v)
    d1 = _conv(sd, "reduce_chan_level1", torch.cat([_up(sd, "up2_1", d2), e1], 1))
    d1, k, v = _level(sd, arch, "decoder_level1", d1, k_cached[7], v_cached[7]); ks.append(k); vs.append(v)
    r, _, _ = _level(sd, arch, "refinement", d1)
    out = _conv(sd, "ending", r, 1, 1) + current
    return out[:, :, :h, :w], ks, vs


def run_clip(sd: SD, opt: dict, clip: Tensor, sr: bool = False):
    """Causal frame loop of video_restoration_model.py:85-92: frame j sees [clip[j-1 or 0], clip[j]]."""
    kc = vc = None
    outs, caches = [], []
    for j in range(clip.shape[1]):
        x = torch.stack([clip[:, max(j - 1, 0)], clip[:, j]], dim=1)
        o, kc, vc = turtle_forward(sd, opt, x, kc, vc, sr=sr)
        outs.append(o)
        caches.append((kc, vc))
    return outs, caches
