"""Deterministic synthetic weights and frames shared by the fixtures, the tests and the bench.

No trained Turtle checkpoint is reachable offline, so parity is weight-agnostic:
the reference, the oracle and the HIP path all run on the SAME weights, produced here from a
counter-based PRNG that any side can re-implement independently:

* stream for tensor ``name``: ``splitmix64(crc32(name) ^ seed, i)`` for element ``i`` (C order),
  mapped to ``u = 2*((x >> 11) * 2**-53) - 1`` in [-1, 1);
* conv weight / bias: ``u / sqrt(fan_in)`` (the PyTorch default-init bound, fan_in of the weight);
* LayerNorm weight ``1 + 0.1u``, bias ``0.02u``;
* ReducedAttn ``beta`` / FeedForward ``gamma``: ``0.1u`` (the reference initialises them to zero,
  turtle_t1_arch.py:202,734, which would make those blocks identically zero);
* attention ``temperature``: ``1 + 0.25(u + 1)``.

Frames are uniform [0, 1) from the stream named ``frames``.
"""
from __future__ import annotations

import zlib

import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix_uniform(name: str, n: int, seed: int = 0) -> np.ndarray:
    """``n`` float64 values in [-1, 1) from the counter-based splitmix64 stream of ``name``."""
    base = np.uint64((zlib.crc32(name.encode()) ^ seed) & 0xFFFFFFFFFFFFFFFF)
    with np.errstate(over="ignore"):
        i = np.arange(1, n + 1, dtype=np.uint64)
        z = base + i * _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    u = (z >> np.uint64(11)).astype(np.float64) * (2.0 ** -53)
    return 2.0 * u - 1.0


def param_value(name: str, shape, seed: int = 0, fan_in_of=None) -> np.ndarray:
    """Synthetic float32 value for state-dict entry ``name`` of ``shape``.

    ``fan_in_of`` maps a bias name to the shape of its conv weight (needed for the bias bound).
    """
    n = int(np.prod(shape)) if len(shape) else 1
    u = splitmix_uniform(name, n, seed)
    leaf = name.rsplit(".", 1)[-1]
    if len(shape) == 1 and name.rsplit(".", 2)[-2] == "body":     # LayerNorm body.weight/bias
        v = 1.0 + 0.1 * u if leaf == "weight" else 0.02 * u
    elif leaf in ("beta", "gamma"):
        v = 0.1 * u
    elif leaf == "temperature":
        v = 1.0 + 0.25 * (u + 1.0)
    elif leaf == "weight" and len(shape) == 4:
        fan_in = shape[1] * shape[2] * shape[3]
        v = u / np.sqrt(fan_in)
    elif leaf == "bias":
        wshape = fan_in_of(name) if fan_in_of is not None else None
        if wshape is None:
            raise KeyError(f"no weight shape for bias {name}")
        fan_in = wshape[1] * wshape[2] * wshape[3]
        v = u / np.sqrt(fan_in)
    else:
        raise KeyError(f"no synthetic rule for {name} {tuple(shape)}")
    return v.astype(np.float32).reshape(shape)


def synthetic_state_dict(shapes: dict, seed: int = 0) -> dict:
    """``{name: float32 ndarray}`` for every ``name -> shape`` entry of a Turtle state dict."""
    def fan_in_of(bias_name):
        w = bias_name[: -len("bias")] + "weight"
        return shapes.get(w)

    return {k: param_value(k, tuple(s), seed, fan_in_of) for k, s in shapes.items()}


def synthetic_frames(shape, seed: int = 0, name: str = "frames") -> np.ndarray:
    """Uniform [0, 1) float32 frames, e.g. ``shape = (B, T, 3, H, W)``."""
    n = int(np.prod(shape))
    u = splitmix_uniform(name, n, seed)
    return ((u + 1.0) * 0.5).astype(np.float32).reshape(shape)


def causal_pairs(clip: np.ndarray, j: int) -> np.ndarray:
    """``[B, 2, C, H, W]`` input of frame ``j``: ``[clip[:, j-1 or 0], clip[:, j]]``.

    Frame 0 uses itself as the previous frame (video_restoration_model.py:89,
    inference.py:281-282).
    """
    prev = clip[:, max(j - 1, 0)]
    return np.stack([prev, clip[:, j]], axis=1)
