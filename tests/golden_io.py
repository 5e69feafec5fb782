"""Helpers to read the committed golden vectors (data only, allow_pickle=False)."""
import json
import os

import numpy as np
import torch

from turtlevsr_amd.synthetic import synthetic_state_dict

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    arr = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    with open(os.path.join(GOLDEN, name + ".json")) as f:
        meta = json.load(f)
    return {k: arr[k] for k in arr.files}, meta


def key_shapes(model="Turtle_t1"):
    with open(os.path.join(GOLDEN, "state_dict_keys.json")) as f:
        return {k: tuple(s) for k, s in json.load(f)[model]}


def tiny_shapes_from_opt(opt):
    """Shapes of a Turtle_t1 state dict for an arbitrary opt, built by our own parameter holder."""
    from turtlevsr_amd.model import TurtleParams
    return {k: tuple(v.shape) for k, v in TurtleParams(opt).state_dict().items()}


def synth_sd(shapes, seed):
    return {k: torch.from_numpy(v) for k, v in synthetic_state_dict(shapes, seed).items()}


def check_summary(rec, key, t, rtol=1e-4, atol=1e-5):
    """Compare a tensor against the checksum + samples stored by gen_golden.summary()."""
    a = t.detach().double().reshape(-1).cpu().numpy()
    assert tuple(rec[key + "__shape"]) == tuple(t.shape), (key, tuple(t.shape))
    samp = a[rec[key + "__idx"]]
    np.testing.assert_allclose(samp, rec[key + "__samp"], rtol=rtol, atol=atol, err_msg=key)
    np.testing.assert_allclose(a.sum(), rec[key + "__sum"], rtol=1e-4, atol=atol * a.size ** 0.5, err_msg=key)
    np.testing.assert_allclose(np.abs(a).sum(), rec[key + "__abssum"], rtol=1e-4, err_msg=key)


def clip_input(g, meta):
    """The clip a golden file was generated from: stored (`clip`) for small inputs, else regenerated
    with the same deterministic generator and checked against the stored checksum."""
    if "clip" in g:
        return g["clip"]
    from turtlevsr_amd.synthetic import synthetic_frames
    clip = synthetic_frames(tuple(meta["shape"]), meta["seed"], name="frames")
    np.testing.assert_allclose(clip.astype(np.float64).sum(), meta["clip_sum"], rtol=1e-12)
    return clip


def check_out(g, j, o, atol, rtol):
    """Frame j's output against the golden record: in full where stored (max-abs <= atol, no
    relative slack), else checksum + samples (atol, rtol)."""
    o = o.detach().cpu() if torch.is_tensor(o) else torch.from_numpy(np.asarray(o))
    key = f"out{j}"
    if key in g:
        np.testing.assert_allclose(o.numpy(), g[key], atol=atol, rtol=0, err_msg=key)
        return float(np.abs(o.numpy() - g[key]).max())
    check_summary(g, key, o, rtol=rtol, atol=atol)
    return None
