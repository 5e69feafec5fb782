"""Parameter holders with the reference's module paths, so ``state_dict()`` has the same 633 keys.

These modules hold ``nn.Parameter`` tensors only; they compute nothing. The inference forward
lives in the HIP library (``turtlevsr_amd/model.py`` drives ``libturtle_hip.so`` through
``_lib.py``); the training graph over the same tree is ``turtlevsr_amd/train.py``. Module / parameter names and registration order follow the
reference constructors so ``load_state_dict(torch.load(p)['params'], strict=True)`` of a reference
checkpoint works unchanged (base_model.py:261-286, inference.py:248-255):

* LayerNorm ``normX.body.weight`` (+ ``.bias`` for WithBias)         turtle_t1_arch.py:67-112
* ReducedAttn ``beta, conv1, conv2, conv3``                         704-742
* FeedForward ``gamma, conv4, conv5``                               181-210
* GatedFeedForward ``project_in, dwconv, project_out``               159-178
* ChannelAttention / FrameHistoryRouter ``temperature, qkv, qkv_dwconv, project_out``   666-702 / 218-286
* CausalHistoryModel ``spatial_aligner.*, ChanAttn.*, kv, kv_dwconv``                     612-662
* StateAlignBlock ``temperature, qk, qk_dwconv, v, v_dwconv, k2, k2_dwconv, q2, q2_dwconv,
  project_out``                                                      289-316
* Down/Upsample ``body.0``                                          136-154
"""
from __future__ import annotations

import torch
import torch.nn as nn

from .arch import BlockSpec, TurtleArch, resolve


def _conv(cin, cout, k=1, groups=1, bias=False):
    return nn.Conv2d(cin, cout, k, padding=k // 2 if k == 3 else 0, groups=groups, bias=bias)


class _LNBody(nn.Module):
    def __init__(self, c, ln_type):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(c))
        if ln_type != "BiasFree":
            self.bias = nn.Parameter(torch.zeros(c))


class LayerNormParams(nn.Module):
    def __init__(self, c, ln_type):
        super().__init__()
        self.body = _LNBody(c, ln_type)


class ReducedAttnParams(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv1 = _conv(c, 2 * c, bias=True)
        self.conv2 = _conv(2 * c, 2 * c, 3, groups=2 * c, bias=True)
        self.conv3 = _conv(2 * c, c, bias=True)
        self.beta = nn.Parameter(torch.zeros(1, c, 1, 1))


class FeedForwardParams(nn.Module):
    def __init__(self, c):
        super().__init__()
        self.conv4 = _conv(c, 2 * c, bias=True)
        self.conv5 = _conv(2 * c, c, bias=True)
        self.gamma = nn.Parameter(torch.zeros(1, c, 1, 1))


class GatedFFNParams(nn.Module):
    def __init__(self, c, hidden, bias):
        super().__init__()
        self.project_in = _conv(c, 2 * hidden, bias=bias)
        self.dwconv = _conv(2 * hidden, 2 * hidden, 3, groups=2 * hidden, bias=bias)
        self.project_out = _conv(hidden, c, bias=bias)


class ChannelAttnParams(nn.Module):
    """Shared by ChannelAttention and FrameHistoryRouter (identical parameter sets)."""

    def __init__(self, c, heads, bias):
        super().__init__()
        self.temperature = nn.Parameter(torch.ones(heads, 1, 1))
        self.qkv = _conv(c, 3 * c, bias=bias)
        self.qkv_dwconv = _conv(3 * c, 3 * c, 3, groups=3 * c, bias=bias)
        self.project_out = _conv(c, c, bias=bias)


class StateAlignParams(nn.Module):
    def __init__(self, c, ws, bias):
        super().__init__()
        self.temperature = nn.Parameter(torch.ones(1, 1, 1))
        self.qk = _conv(c, 2 * c, bias=bias)
        self.qk_dwconv = _conv(2 * c, 2 * c, 3, groups=2 * c, bias=bias)
        self.v = _conv(c, c, bias=bias)
        self.v_dwconv = _conv(c, c, 3, groups=c, bias=bias)
        self.k2 = _conv(c, 2 * c, bias=bias)
        self.k2_dwconv = nn.Conv2d(2 * c, 2 * c, ws, stride=ws, padding=1, groups=2 * c, bias=bias)
        self.q2 = _conv(c, 2 * c, bias=bias)
        self.q2_dwconv = nn.Conv2d(2 * c, 2 * c, ws, stride=ws, padding=1, groups=2 * c, bias=bias)
        self.project_out = _conv(c, c, bias=bias)


class CausalHistoryParams(nn.Module):
    def __init__(self, c, heads, ws, bias):
        super().__init__()
        self.spatial_aligner = StateAlignParams(c, ws, bias)
        self.ChanAttn = ChannelAttnParams(c, heads, bias)
        self.kv = _conv(c, 2 * c, bias=bias)
        self.kv_dwconv = _conv(2 * c, 2 * c, 3, groups=2 * c, bias=bias)


class BlockParams(nn.Module):
    def __init__(self, spec: BlockSpec, ln_type: str, bias: bool):
        super().__init__()
        c = spec.dim
        self.norm1 = LayerNormParams(c, ln_type)
        if spec.attn == "ReducedAttn":
            self.attn = ReducedAttnParams(c)
        elif spec.attn in ("Channel", "FHR"):
            self.attn = ChannelAttnParams(c, spec.heads, bias)
        elif spec.attn == "CHM":
            self.attn = CausalHistoryParams(c, spec.heads, spec.ws, bias)
        else:
            self.attn = None
        self.norm2 = LayerNormParams(c, ln_type)
        self.ffn = GatedFFNParams(c, spec.hidden, bias) if spec.ffn == "GFFW" else FeedForwardParams(c)


class LevelParams(nn.Module):
    def __init__(self, blocks, ln_type, bias):
        super().__init__()
        self.transformer_blocks = nn.ModuleList([BlockParams(b, ln_type, bias) for b in blocks])


class _Resample(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.body = nn.Sequential(_conv(cin, cout, 3))


class TurtleParams(nn.Module):
    """The full Turtle_t1 parameter tree (turtle_t1_arch.py:932-1043)."""

    def __init__(self, opt_or_arch):
        super().__init__()
        a = opt_or_arch if isinstance(opt_or_arch, TurtleArch) else resolve(opt_or_arch)
        self.arch = a
        d, lv = a.dim, a.levels
        self.input_projection = _conv(a.in_ch, d, 3, bias=a.bias)
        self.encoder_level1 = LevelParams(lv["encoder_level1"].blocks, a.ln_type, a.bias)
        self.down1_2 = _Resample(d, d // 2)
        self.encoder_level2 = LevelParams(lv["encoder_level2"].blocks, a.ln_type, a.bias)
        self.down2_3 = _Resample(2 * d, d)
        self.encoder_level3 = LevelParams(lv["encoder_level3"].blocks, a.ln_type, a.bias)
        self.down3_4 = _Resample(4 * d, 2 * d)
        self.latent = LevelParams(lv["latent"].blocks, a.ln_type, a.bias)
        self.up4_3 = _Resample(8 * d, 16 * d)
        self.reduce_chan_level3 = _conv(8 * d, 4 * d, bias=a.bias)
        self.decoder_level3 = LevelParams(lv["decoder_level3"].blocks, a.ln_type, a.bias)
        self.up3_2 = _Resample(4 * d, 8 * d)
        self.reduce_chan_level2 = _conv(4 * d, 2 * d, bias=a.bias)
        self.decoder_level2 = LevelParams(lv["decoder_level2"].blocks, a.ln_type, a.bias)
        self.up2_1 = _Resample(2 * d, 4 * d)
        self.reduce_chan_level1 = _conv(2 * d, d, bias=a.bias)
        self.decoder_level1 = LevelParams(lv["decoder_level1"].blocks, a.ln_type, a.bias)
        self.refinement = LevelParams(lv["refinement"].blocks, a.ln_type, a.bias)
        self.ending = _conv(d, a.out_ch, 3, bias=True)
