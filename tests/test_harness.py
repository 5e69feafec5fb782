"""Evaluation harness (turtlevsr_amd/harness.py): tiling, overlap
averaging, per-tile cache threading, uint8 PSNR / SSIM and the checkpoint loader, on CPU with stub
models and the oracle; the HIP module through the harness is in the gpu-marked test at the end."""
import math
import os

import numpy as np
import pytest
import torch

from turtlevsr_amd.harness import (bgr2ycbcr, calc_PSNR, load_checkpoint, pad_to_multiple, run_inference_patched,
                                   run_video, ssim_calculate, tensor2img, tile_starts)


def test_tile_starts_cover_and_stay_inside():
    assert tile_starts(64, 64, 32) == [0]
    assert tile_starts(100, 64, 32) == [0, 32, 36]
    assert tile_starts(320, 128, 64) == [0, 64, 128, 192]
    for size, tile, ov in [(136, 64, 16), (1088, 320, 128), (544, 320, 192), (96, 32, 8)]:
        st = tile_starts(size, tile, tile - ov)
        assert st[0] == 0 and st[-1] == size - tile
        covered = np.zeros(size, bool)
        for s in st:
            covered[s:s + tile] = True
        assert covered.all()


def test_pad_to_multiple_reflect():
    x = torch.arange(2 * 3 * 37 * 50, dtype=torch.float32).reshape(2, 3, 37, 50)
    y = pad_to_multiple(x, 8)
    assert y.shape == (2, 3, 40, 56)
    assert torch.equal(y[..., :37, :50], x)
    assert torch.equal(y[..., 37, :50], x[..., 35, :])        # reflect (edge not repeated)
    z = torch.zeros(1, 3, 40, 48)
    assert pad_to_multiple(z, 8) is z


class _Identity:
    """model(x, k, v): returns the current frame; the cache counts calls per tile."""

    def __call__(self, x, k, v):
        n = 1 if k is None else int(k[0].item()) + 1
        return x[:, 1].clone(), [torch.tensor(float(n))] + [None] * 7, [None] * 8


def test_patched_identity_and_cache_threading():
    torch.manual_seed(0)
    prev, cur = torch.rand(1, 3, 45, 70), torch.rand(1, 3, 45, 70)
    m = _Identity()
    out, pk, pv = run_inference_patched(prev, cur, m, tile=32, tile_overlap=8)
    padded = pad_to_multiple(cur, 8)
    assert out.shape == padded.shape
    assert torch.allclose(out, padded.clamp(0, 1), atol=1e-6)      # overlaps average identical values
    keys = {f"{h}-{w}" for h in tile_starts(48, 32, 24) for w in tile_starts(72, 32, 24)}
    assert set(pk) == keys and set(pv) == keys
    for _ in range(2):
        out, pk, pv = run_inference_patched(prev, cur, m, 32, 8, pk, pv)
    assert all(int(v[0].item()) == 3 for v in pk.values())


def test_patched_overlap_average():
    """Outputs that differ per tile are averaged where tiles overlap (E / W)."""
    calls = []

    def m(x, k, v):
        calls.append(1)
        return torch.full_like(x[:, 1], float(len(calls))), [None] * 8, [None] * 8

    out, _, _ = run_inference_patched(torch.zeros(1, 1, 16, 24), torch.zeros(1, 1, 16, 24), m, tile=16, tile_overlap=8)
    # w tiles at 0 and 8 (values 1 and 2): columns 8..15 are their mean, clamped to [0, 1]
    assert torch.allclose(out[..., :8], torch.ones(1)) and torch.allclose(out[..., 8:16], torch.ones(1))
    out2, _, _ = run_inference_patched(torch.zeros(1, 1, 16, 24), torch.zeros(1, 1, 16, 24),
                                       lambda x, k, v: (x[:, 1] + 0.25 * (x.shape[-1] > 0), None, None), 16, 8)
    assert torch.allclose(out2, torch.full_like(out2, 0.25))
    with pytest.raises(ValueError):
        run_inference_patched(torch.zeros(1, 1, 20, 20), torch.zeros(1, 1, 20, 20), m, tile=12, tile_overlap=4)


def test_psnr_ssim_ycbcr():
    a = np.full((8, 8, 3), 100, np.uint8)
    assert calc_PSNR(a, a) == float("inf")
    assert calc_PSNR(a, a + 1) == pytest.approx(20 * math.log10(255.0))
    assert ssim_calculate(a, a) == pytest.approx(1.0)
    white = np.full((2, 2, 3), 255, np.uint8)
    black = np.zeros((2, 2, 3), np.uint8)
    assert int(bgr2ycbcr(white)[0, 0]) == 235 and int(bgr2ycbcr(black)[0, 0]) == 16
    t = torch.tensor([[[0.0, 0.5], [1.0, 1.2]]] * 3)
    img = tensor2img(t)
    assert img.dtype == np.uint8 and img.shape == (2, 2, 3)
    assert img[0, 0, 0] == 0 and img[0, 1, 0] == 128 and img[1, 1, 0] == 255    # rounded, clamped


def test_run_video_whole_and_tiled_identity():
    torch.manual_seed(1)
    frames = [torch.rand(3, 40, 56) for _ in range(3)]
    whole = run_video(frames, frames, _Identity())
    tiled = run_video(frames, frames, _Identity(), tile=32, tile_overlap=16)
    assert whole.psnr == [float("inf")] * 3 and tiled.psnr == [float("inf")] * 3
    assert tiled.ssim[0] == pytest.approx(1.0)


def test_load_checkpoint_strips_module_prefix(tmp_path):
    src = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 1), torch.nn.Conv2d(4, 2, 3))
    path = os.path.join(tmp_path, "ck.pth")
    torch.save({"params": {"module." + k: v for k, v in src.state_dict().items()}}, path)
    dst = torch.nn.Sequential(torch.nn.Conv2d(3, 4, 1), torch.nn.Conv2d(4, 2, 3))
    load_checkpoint(dst, path)
    for (k, a), (_, b) in zip(src.state_dict().items(), dst.state_dict().items()):
        assert torch.equal(a, b), k
    torch.save({"params": {"x": torch.zeros(1)}}, path)
    with pytest.raises(RuntimeError):
        load_checkpoint(dst, path)


def test_y_channel_psnr_follows_reference_conversion():
    """Y-channel PSNR builds its uint8 images like inference.py:314-319: (x*255).astype(uint8),
    truncating, no clamp (the RGB path rounds through tensor2img instead)."""
    gt = torch.full((3, 4, 4), 0.5)               # 127.5 -> 127 truncated (128 rounded)
    out = torch.full((3, 4, 4), 0.5)
    out[:, 0, 0] = 0.503                          # 128.27 -> 128
    res = run_video([out], [gt], lambda x, k, v: (x[:, 1], [None] * 8, [None] * 8), y_channel_PSNR=True)
    g8 = (gt * 255.0).permute(1, 2, 0).numpy().astype(np.uint8)
    o8 = (out * 255.0).permute(1, 2, 0).numpy().astype(np.uint8)
    want = calc_PSNR(bgr2ycbcr(o8[:, :, ::-1]), bgr2ycbcr(g8[:, :, ::-1]))
    assert res.psnr[0] == pytest.approx(want)
    assert int(g8[0, 0, 0]) == 127 and int(o8[0, 0, 0]) == 128


def test_load_checkpoint_full_turtle_state_dict(tmp_path):
    """A reference-style GoPro checkpoint ({'params': state_dict} with the DDP `module.` prefix,
    base_model.py:194-224) loads strictly into the HIP module: all 633 keys, values unchanged."""
    import yaml
    from golden_io import synth_sd
    from turtlevsr_amd.model import TurtleHIP
    with open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "options",
                           "Turtle_Deblur_Gopro.yml")) as f:
        opt = yaml.safe_load(f)
    m = TurtleHIP(opt)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    assert len(shapes) == 633
    sd = synth_sd(shapes, 3)
    path = os.path.join(tmp_path, "net_g_latest.pth")
    torch.save({"params": {"module." + k: v for k, v in sd.items()}}, path)
    load_checkpoint(m, path)
    for k, v in m.state_dict().items():
        assert torch.equal(v, sd[k]), k
    torch.save({"params": {"module." + k: v for k, v in list(sd.items())[:-1]}}, path)
    with pytest.raises(RuntimeError):
        load_checkpoint(TurtleHIP(opt), path)


def test_cache_shapes_are_checked_against_the_frame():
    """Incoming caches must match this frame's batch / size up to their temporal extent (the
    kernels index them with the frame's dimensions)."""
    from turtlevsr_amd.model import TurtleHIP
    kind = [0, 0, 0, 1, 0, 2, 0, 0]
    ks = [(1,) * 5] * 3 + [(2, 8, 128, 1024, 1)] + [(1,) * 5] + [(2, 2, 1, 256, 512)] + [(1,) * 5] * 2
    vs = [(1,) * 5] * 5 + [(2, 2, 1, 256, 4096)] + [(1,) * 5] * 2
    t_in = [0, 0, 0, 64, 0, 1, 0, 0]
    kc = [None] * 8
    vc = [None] * 8
    kc[3] = vc[3] = torch.empty(2, 8, 64, 1024)
    kc[5], vc[5] = torch.empty(2, 1, 1, 256, 512), torch.empty(2, 1, 1, 256, 4096)
    TurtleHIP._check_caches(kind, ks, vs, t_in, kc, vc)
    bad = list(kc)
    bad[5] = torch.empty(2, 1, 1, 64, 512)           # caches of a smaller frame
    with pytest.raises(ValueError):
        TurtleHIP._check_caches(kind, ks, vs, t_in, bad, vc)
    bad = list(kc)
    bad[3] = torch.empty(1, 8, 64, 1024)             # another batch size
    with pytest.raises(ValueError):
        TurtleHIP._check_caches(kind, ks, vs, t_in, bad, vc)
    bad = list(vc)
    bad[5] = None
    with pytest.raises(ValueError):
        TurtleHIP._check_caches(kind, ks, vs, t_in, kc, bad)


def _oracle_model(meta):
    from golden_io import synth_sd
    from oracle import turtle_ref as R
    from turtlevsr_amd.model import TurtleHIP
    shapes = {k: tuple(v.shape) for k, v in TurtleHIP(meta["opt"]).state_dict().items()}
    sd = synth_sd(shapes, meta["seed"])

    def m(x, k, v):
        return R.turtle_forward(sd, meta["opt"], x, k, v)
    return m, sd


def test_oracle_through_tiled_harness():
    from golden_io import load
    _, meta = load("clip_tiny_64")
    m, _ = _oracle_model(meta)
    torch.manual_seed(2)
    frames = [torch.rand(3, 70, 100) for _ in range(2)]   # padded 72 x 104: 2 x 2 tiles of 64 (N = 16 >= top-5)
    r = run_video(frames, frames, m, tile=64, tile_overlap=16, keep_outputs=True)
    assert len(r.psnr) == 2 and all(np.isfinite(p) for p in r.psnr)
    assert r.outputs[0].shape == (3, 70, 100) and float(r.outputs[1].min()) >= 0 and float(r.outputs[1].max()) <= 1


@pytest.mark.gpu
def test_hip_vs_oracle_through_tiled_harness():
    """The HIP module through the tiled harness (per-tile caches on the GPU) against the oracle
    through the same harness: fp32 restored frames agree to 1e-4 (uint8 PSNR identical or inf)."""
    from golden_io import load
    from turtlevsr_amd.model import TurtleHIP
    _, meta = load("clip_tiny_64")
    m_ref, sd = _oracle_model(meta)
    hip = TurtleHIP(meta["opt"], dtype="fp32")
    hip.load_state_dict(sd, strict=True)
    hip = hip.cuda().eval()
    torch.manual_seed(3)
    frames = [torch.rand(3, 70, 100) for _ in range(3)]
    with torch.no_grad():
        r_ref = run_video(frames, frames, m_ref, tile=64, tile_overlap=16, keep_outputs=True)
        r_hip = run_video([f.cuda() for f in frames], frames, hip, tile=64, tile_overlap=16, keep_outputs=True)
    for a, b in zip(r_hip.outputs, r_ref.outputs):
        assert float((a - b).abs().max()) <= 1e-4
    for a, b in zip(r_hip.psnr, r_ref.psnr):
        assert abs(a - b) <= 0.05 or (math.isinf(a) and math.isinf(b))


@pytest.mark.gpu
def test_hip_vs_oracle_published_tiled_protocol():
    """The reference's published evaluation protocol on the HIP path (basicsr/inference.py:590-609,
    172-246): GoPro widths, tile 320, overlap 192, per-tile caches carried through HOST memory
    between frames (:227-237). 3 frames of 352 x 480 = 2 x 3 tiles per frame. fp32 HIP vs the
    oracle through the same harness: restored frames to 2e-4, uint8 PSNR within 0.01 dB."""
    from golden_io import load
    from turtlevsr_amd.model import TurtleHIP
    _, meta = load("clip_gopro_64")
    m_ref, sd = _oracle_model(meta)
    hip = TurtleHIP(meta["opt"], dtype="fp32")
    hip.load_state_dict(sd, strict=True)
    hip = hip.cuda().eval()
    torch.manual_seed(4)
    frames = [torch.rand(3, 352, 480) for _ in range(3)]
    with torch.no_grad():
        r_ref = run_video(frames, frames, m_ref, tile=320, tile_overlap=192, keep_outputs=True)
        r_hip = run_video([f.cuda() for f in frames], frames, hip, tile=320, tile_overlap=192, keep_outputs=True,
                          cache_device="cpu")
    for a, b in zip(r_hip.outputs, r_ref.outputs):
        assert float((a.cpu() - b).abs().max()) <= 2e-4
    for a, b in zip(r_hip.psnr, r_ref.psnr):
        assert abs(a - b) <= 0.01 or (math.isinf(a) and math.isinf(b))
