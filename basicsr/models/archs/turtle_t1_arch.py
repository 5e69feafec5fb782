"""Drop-in replacement for basicsr/models/archs/turtle_t1_arch.py (GoPro / VRDS arch).

``make_model(opt)`` (turtle_t1_arch.py:10-53) returns a module with the same state_dict and the
same ``forward(inp_img_, k_cached=None, v_cached=None)`` contract (1045-1132), executed by the
MI355X HIP library (turtlevsr_amd/csrc, include/turtle_hip.h).
"""
from importlib import import_module

from turtlevsr_amd.model import TurtleHIP


class Turtle_t1(TurtleHIP):
    def __init__(self, opt: dict, dtype: str = "fp32"):
        super().__init__(opt, sr=False, dtype=dtype, t0=False)


def make_model(opt):
    return Turtle_t1(opt, dtype=opt.get("hip_dtype", "fp32"))


def create_video_model(opt):
    """turtle_t1_arch.py:56-59."""
    return import_module("basicsr.models.archs.turtle_t1_arch").make_model(opt)
