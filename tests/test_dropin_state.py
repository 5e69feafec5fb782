"""Drop-in module state handling on the MI355X, through the C ABI:

* SAB history arena (model.py _sab_out): at B = 1 a frame's returned SAB caches are views whose
  kept frames are the incoming cache's own frames (no roll copy in the library), yet every
  returned history stays immutable - a caller re-running from an older cache (a branched history,
  as the tiled harness's per-tile caches or a restart would) gets the same result as from a private
  copy of that cache (reference semantics: torch.cat builds a fresh tensor, turtle_t1_arch.py:581,
  610);
* minimum input size: a 32x32 frame has N = 4 SAB tokens and the
  reference's topk(k=5) raises "selected index k out of range" (turtle_t1_arch.py:404); the library
  refuses it the same way (TURTLE_EINVAL, RuntimeError), 32x64 (N = 8) runs;
* parameter rebinding: load_state_dict(assign=True) replaces the Parameter objects; a
  train step on the new objects and the eval() forward after it must see the updated weights.
"""
import pytest
import torch

from golden_io import load, synth_sd

pytestmark = pytest.mark.gpu


def _model(opt, seed, dtype):
    from turtlevsr_amd.model import TurtleHIP
    m = TurtleHIP(opt, dtype=dtype)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    m.load_state_dict(synth_sd(shapes, seed), strict=True)
    return m.cuda().eval()


def _pair(clip, j):
    return torch.stack([clip[:, max(j - 1, 0)], clip[:, j]], dim=1).contiguous()


@pytest.mark.parametrize("dtype", ["fp32", "bf16"])
def test_sab_arena_zero_copy_and_immutable_history(dtype):
    from turtlevsr_amd.synthetic import synthetic_frames
    _, meta = load("clip_gopro_64")
    clip = torch.from_numpy(synthetic_frames((1, 7, 3, 128, 128), 41)).cuda()
    m = _model(meta["opt"], meta["seed"], dtype)
    hist = []
    kc = vc = None
    with torch.no_grad():
        for j in range(6):
            o, kc, vc = m(_pair(clip, j), kc, vc)
            hist.append((o.clone(), list(kc), list(vc)))
        # steady state: slot 5 (dec3, ntc 3) of frame 5 starts one frame after frame 4's in the same
        # storage - the kept frames were not copied
        k4, k5 = hist[4][1][5], hist[5][1][5]
        assert k5.untyped_storage().data_ptr() == k4.untyped_storage().data_ptr()
        fb = k4[0, 0].numel() * k4.element_size()
        assert k5.data_ptr() == k4.data_ptr() + fb
        # branch: re-run frame 5 from frame 4's (arena-view) history and from a private copy of it
        k_old, v_old = hist[4][1], hist[4][2]
        snap = [None if t is None else t.clone() for t in k_old + v_old]
        o_a, ka, va = m(_pair(clip, 5), k_old, v_old)
        o_b, kb, vb = m(_pair(clip, 5), [None if t is None else t.clone() for t in k_old],
                        [None if t is None else t.clone() for t in v_old])
        assert torch.equal(o_a, hist[5][0]) and torch.equal(o_b, hist[5][0])
        for a, b, c in zip(ka + va, kb + vb, hist[5][1] + hist[5][2]):
            if c is not None:
                assert torch.equal(a, b) and torch.equal(a, c)
        # the older history was not overwritten by any of the later frames
        for t, s in zip(k_old + v_old, snap):
            if s is not None:
                assert torch.equal(t, s)
        # continuing the first line of history after the branch still matches the copy-based run
        o6, _, _ = m(_pair(clip, 6), hist[5][1], hist[5][2])
        o6b, _, _ = m(_pair(clip, 6), [None if t is None else t.clone() for t in hist[5][1]],
                      [None if t is None else t.clone() for t in hist[5][2]])
        assert torch.equal(o6, o6b)


def test_sab_arena_refill_matches_roomy_arena():
    """An exhausted arena is replaced by a fresh one that the library fills by copying the kept
    frames (turtle.cpp sab_cache_shift): a 1-frame-headroom arena, refilled every other frame, gives
    the same frames bit for bit as the default (byte-budgeted, never refilled here) arena."""
    from turtlevsr_amd.synthetic import synthetic_frames
    _, meta = load("clip_gopro_64")
    clip = torch.from_numpy(synthetic_frames((1, 9, 3, 128, 128), 43)).cuda()
    outs = []
    for tight in (False, True):
        m = _model(meta["opt"], meta["seed"], "bf16")
        if tight:
            m._ARENA_EXTRA, m._ARENA_BYTES = 1, 0
        kc = vc = None
        res = []
        with torch.no_grad():
            for j in range(9):
                o, kc, vc = m(_pair(clip, j), kc, vc)
                res.append(o.clone())
        outs.append(res)
    for a, b in zip(*outs):
        assert torch.equal(a, b)


def test_minimum_input_size_is_refused():
    _, meta = load("clip_gopro_64")
    m = _model(meta["opt"], meta["seed"], "bf16")
    with torch.no_grad():
        x = torch.rand(1, 2, 3, 32, 32, device="cuda")
        with pytest.raises(RuntimeError, match="selected index k out of range"):
            m(x)
        o, _, _ = m(torch.rand(1, 2, 3, 32, 64, device="cuda"))
        assert o.shape == (1, 3, 32, 64) and torch.isfinite(o).all()


def test_assign_load_then_train_step_then_eval_uses_new_weights():
    from turtlevsr_amd.synthetic import synthetic_frames
    _, meta = load("train_tiny")
    m = _model(meta["opt"], meta["seed"], "fp32")
    x = torch.from_numpy(synthetic_frames((1, 2, 3, 64, 64), 43)).cuda()
    with torch.no_grad():
        m(x)                                            # packs and records the signature
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    sd = {k: v.cuda() for k, v in synth_sd(shapes, meta["seed"] + 7).items()}
    m.load_state_dict(sd, strict=True, assign=True)     # new Parameter objects
    with torch.no_grad():
        m(x)                                            # repack: the signature must follow the new objects
    for p in m.parameters():
        p.requires_grad_(True)
    m.train()
    out, _, _ = m(x)
    out.abs().mean().backward()
    opt = torch.optim.SGD(m.parameters(), lr=1e-2)
    opt.step()
    m.eval()
    with torch.no_grad():
        got, _, _ = m(x)
    ref = _model(meta["opt"], meta["seed"], "fp32")
    ref.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()}, strict=True)
    with torch.no_grad():
        want, _, _ = ref(x)
    assert torch.equal(got, want), float((got - want).abs().max())


def test_tiled_harness_keeps_one_small_arena_per_tile():
    """the tiled protocol (harness.run_inference_patched, inference.py:172-246)
    runs one B = 1 stream per tile position, interleaved frame by frame. Each stream keeps its own
    SAB arena (a hit every frame: no roll copy), sized small (tnew + 6 frames within 6 frames), and
    device memory stays flat from frame to frame instead of a full-budget arena per tile and call."""
    from turtlevsr_amd.harness import run_video
    from turtlevsr_amd.synthetic import synthetic_frames
    _, meta = load("clip_gopro_64")
    m = _model(meta["opt"], meta["seed"], "bf16")
    clip = torch.from_numpy(synthetic_frames((1, 6, 3, 128, 192), 47))[0].cuda()
    frames = [clip[j] for j in range(6)]
    mem = []

    class Probe:
        def __call__(self, x, k, v):
            return m(x, k, v)

    with torch.no_grad():
        for n in (3, 6):
            torch.cuda.synchronize()
            run_video(frames[:n], frames[:n], Probe(), tile=64, tile_overlap=16)
            torch.cuda.synchronize()
            mem.append(torch.cuda.memory_allocated())
    ntile = 3 * 4                                   # tile starts: h [0, 48, 64], w [0, 48, 96, 128]
    for slot, streams in m._arenas.items():
        assert len(streams) <= 2 * ntile            # two videos ran; at most one arena per tile each
        for a in streams:
            assert a["extra"] == m._ARENA_EXTRA     # no stream outgrew its first arena in 6 frames
    m.release_history()
    torch.cuda.synchronize()
    assert torch.cuda.memory_allocated() <= mem[-1]
    assert mem[1] < mem[0] + (256 << 20)
