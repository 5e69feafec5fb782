"""Drop-in replacement for basicsr/models/archs/turtlesuper_t1_arch.py (MVSR 4x SR arch).

Same blocks as turtle_t1_arch; the current frame is upsampled 4x (bilinear, align_corners=False)
before the network and is the global residual (turtlesuper_t1_arch.py:976-977, 1049-1071); the
output is [B, C, 4H, 4W].
"""
from turtlevsr_amd.model import TurtleHIP


class TurtleSuper_t1(TurtleHIP):
    def __init__(self, opt: dict, dtype: str = "fp32"):
        super().__init__(opt, sr=True, dtype=dtype, t0=False)


def make_model(opt):
    return TurtleSuper_t1(opt, dtype=opt.get("hip_dtype", "fp32"))
