"""Pin the CPU oracle (oracle/turtle_ref.py) to golden vectors produced by the reference itself.

The vectors were generated in the build container by tests/golden/gen_golden.py, which runs the
reference arch files (loaded by path) on the deterministic synthetic weights.
"""
import numpy as np
import pytest
import torch

from oracle import turtle_ref as R
from golden_io import check_out, check_summary, clip_input, load, synth_sd
from turtlevsr_amd.params import TurtleParams

torch.set_num_threads(8)


def _sd(prefix_shapes, seed):
    return synth_sd(prefix_shapes, seed)


def _block_sd(module_ctor, seed=100):
    m = module_ctor()
    shapes = {"blk." + k: tuple(v.shape) for k, v in m.state_dict().items()}
    return synth_sd(shapes, seed)


def close(a, b, atol=2e-5, rtol=1e-4):
    np.testing.assert_allclose(np.asarray(a), np.asarray(b), atol=atol, rtol=rtol)


def test_layernorm():
    from turtlevsr_amd.params import LayerNormParams
    g, _ = load("block_layernorm")
    x = torch.from_numpy(g["ln_x"])
    sd = _block_sd(lambda: LayerNormParams(64, "WithBias"))
    close(R.layer_norm(sd, "blk", x, "WithBias"), g["ln_y"])
    sd = _block_sd(lambda: LayerNormParams(64, "BiasFree"))
    close(R.layer_norm(sd, "blk", x, "BiasFree"), g["lnbf_y"])


def test_reduced_attn():
    from turtlevsr_amd.params import ReducedAttnParams
    g, _ = load("block_reducedattn")
    sd = _block_sd(lambda: ReducedAttnParams(64))
    close(R.reduced_attn(sd, "blk", torch.from_numpy(g["x"])), g["y"])


def test_ffw():
    from turtlevsr_amd.params import FeedForwardParams
    g, _ = load("block_ffw")
    sd = _block_sd(lambda: FeedForwardParams(128))
    close(R.feed_forward(sd, "blk", torch.from_numpy(g["x"])), g["y"])


def test_gffw():
    from turtlevsr_amd.params import GatedFFNParams
    g, _ = load("block_gffw")
    sd = _block_sd(lambda: GatedFFNParams(256, 640, False))
    close(R.gated_ffn(sd, "blk", torch.from_numpy(g["x"])), g["y"])


def test_channel_attention():
    from turtlevsr_amd.params import ChannelAttnParams
    g, _ = load("block_channel")
    sd = _block_sd(lambda: ChannelAttnParams(256, 4, False))
    close(R.channel_attention(sd, "blk", torch.from_numpy(g["x"]), 4), g["y"])


def test_fhr_with_and_without_cache():
    from turtlevsr_amd.params import ChannelAttnParams
    g, _ = load("block_fhr")
    sd = _block_sd(lambda: ChannelAttnParams(512, 8, False))
    x, kc, vc = (torch.from_numpy(g[k]) for k in ("x", "kc", "vc"))
    y, k, v = R.frame_history_router(sd, "blk", x, 8, 3, kc, vc)
    close(y, g["y"]); close(k, g["k"]); close(v, g["v"])
    y, k, v = R.frame_history_router(sd, "blk", x, 8, 3, None, None)
    close(y, g["y0"]); close(k, g["k0"]); close(v, g["v0"])


def test_state_align_block():
    from turtlevsr_amd.params import StateAlignParams
    g, _ = load("block_sab")
    sd = _block_sd(lambda: StateAlignParams(32, 8, False))
    x, kc, vc = (torch.from_numpy(g[k]) for k in ("x", "kc", "vc"))
    y, k, v = R.state_align(sd, "blk", x, 8, 2, kc, vc)
    close(y, g["y"]); close(k, g["k"]); close(v, g["v"])
    y, k, v = R.state_align(sd, "blk", x, 8, 2, None, None)
    close(y, g["y0"]); close(k, g["k0"]); close(v, g["v0"])


def test_state_align_block_t0():
    """t0 StateAlignBlock (turtle_arch.py:459-533): out = project_out(v) of every frame, k tokens
    from x + positional encoding, dilated and L2-normalised."""
    from turtlevsr_amd.params import StateAlignParams
    g, meta = load("block_sab_t0")
    sd = _block_sd(lambda: StateAlignParams(32, 8, False), seed=meta["seed"])
    x, kc, vc = (torch.from_numpy(g[k]) for k in ("x", "kc", "vc"))
    y, k, v = R.state_align_t0(sd, "blk", x, 8, 2, kc, vc)
    close(y, g["y"]); close(k, g["k"]); close(v, g["v"])
    y, k, v = R.state_align_t0(sd, "blk", x, 8, 2, None, None)
    close(y, g["y0"]); close(k, g["k0"]); close(v, g["v0"])
    with pytest.raises(RuntimeError):                     # < 5 tokens: the discarded top-5 raises
        R.state_align_t0(sd, "blk", x[..., :16, :16], 8, 2, None, None)


def test_causal_history_model():
    from turtlevsr_amd.params import CausalHistoryParams
    g, _ = load("block_chm")
    sd = _block_sd(lambda: CausalHistoryParams(32, 2, 4, False))
    x, kc, vc = (torch.from_numpy(g[k]) for k in ("x", "kc", "vc"))
    y, k, v = R.causal_history(sd, "blk", x, 2, 4, 3, kc, vc)
    close(y, g["y"]); close(k, g["k"]); close(v, g["v"])
    y, k, v = R.causal_history(sd, "blk", x, 2, 4, 3, None, None)
    close(y, g["y0"]); close(k, g["k0"]); close(v, g["v0"])


CLIPS = ["clip_tiny_64", "clip_tiny_ragged", "clip_tiny_both", "clip_tiny_biasfree", "clip_tiny_sr",
         "clip_gopro_64", "clip_tiny_t0", "clip_gopro_t0", "clip_tiny_hetero", "clip_gopro_128x224",
         pytest.param("clip_gopro_256", marks=pytest.mark.slow)]


@pytest.mark.parametrize("name", CLIPS)
def test_clip(name):
    g, meta = load(name)
    opt = meta["opt"]
    shapes = {k: tuple(v.shape) for k, v in TurtleParams(opt).state_dict().items()}
    sd = synth_sd(shapes, meta["seed"])
    clip = torch.from_numpy(clip_input(g, meta))
    outs, caches = R.run_clip(sd, opt, clip, sr=meta["sr"])
    for j, o in enumerate(outs):
        check_out(g, j, o, atol=5e-5, rtol=1e-3)
        kc, vc = caches[j]
        for which, lst in (("k", kc), ("v", vc)):
            for i, t in enumerate(lst):
                key = f"f{j}_{which}{i}"
                if t is None:
                    assert key + "__shape" not in g
                    continue
                check_summary(g, key, t, rtol=1e-3, atol=5e-5)
                if key in g:
                    close(t, g[key], atol=5e-5, rtol=1e-3)


def test_sparse_av_matches_golden_steady_state(monkeypatch):
    """The oracle's sparse A.v switch (SAB_SPARSE_AV, used by the 1080p parity test) computes the same
    frames as the reference: the steady-state 256x256 GoPro golden clip (N = 256 tokens, top-5 keys
    outside the L1 ball exercised) at the dense path's tolerance."""
    monkeypatch.setattr(R, "SAB_SPARSE_AV", True)
    g, meta = load("clip_gopro_256")
    opt = meta["opt"]
    shapes = {k: tuple(v.shape) for k, v in TurtleParams(opt).state_dict().items()}
    sd = synth_sd(shapes, meta["seed"])
    outs, _ = R.run_clip(sd, opt, torch.from_numpy(clip_input(g, meta)), sr=meta["sr"])
    for j, o in enumerate(outs):
        check_out(g, j, o, atol=5e-5, rtol=1e-3)


def test_pad_to_non_square_ragged():
    """check_image_size (turtle_t1_arch.py:1134-1139) pads H and W each to a multiple of 32 with
    zeros at the bottom/right: 540x960 -> 544x960 and 36x70 -> 64x96 (unequal H/W pads)."""
    x = torch.rand(1, 2, 3, 540, 960)
    y = R.pad_to(x)
    assert y.shape[-2:] == (544, 960)
    assert torch.equal(y[..., :540, :], x) and float(y[..., 540:, :].abs().max()) == 0.0
    x = torch.rand(1, 3, 36, 70)
    y = R.pad_to(x)
    assert y.shape[-2:] == (64, 96)
    assert torch.equal(y[..., :36, :70], x)
    assert float(y[..., 36:, :].abs().max()) == 0.0 and float(y[..., :, 70:].abs().max()) == 0.0
