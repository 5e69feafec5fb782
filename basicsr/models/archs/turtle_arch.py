"""Drop-in replacement for basicsr/models/archs/turtle_arch.py (the t0 network, option
``model: Turtle_arch``: Derain / Desnow / NightRain configs).

``make_model(opt)`` (turtle_arch.py:10-53) returns a module with the same state_dict (the t0
StateAlignBlock registers the same parameters as Turtle_t1's, turtle_arch.py:291-316) and the same
``forward(inp_img_, k_cached=None, v_cached=None)`` contract. The t0 aligner discards its attention
(``out = v``, turtle_arch.py:521-523); its caches hold dilated, L2-normalised k tokens
``[B, frames, 1, N, ws*ws*c]`` (turtle_arch.py:480-495) next to the v tokens.
"""
from importlib import import_module

from turtlevsr_amd.model import TurtleHIP


class Turtle(TurtleHIP):
    def __init__(self, opt: dict, dtype: str = "fp32"):
        super().__init__(opt, sr=False, dtype=dtype, t0=True)


def make_model(opt):
    return Turtle(opt, dtype=opt.get("hip_dtype", "fp32"))


def create_video_model(opt):
    """turtle_arch.py:56-59."""
    return import_module("basicsr.models.archs.turtle_arch").make_model(opt)
