"""Run-to-run repeatability of the bf16 forward with each kernel switch (GPU box):
the same frame twice through one module, max |diff| of the outputs."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests"))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
from golden_io import load, synth_sd  # noqa: E402
from turtlevsr_amd.model import TurtleHIP  # noqa: E402
from turtlevsr_amd.synthetic import synthetic_frames  # noqa: E402

_, meta = load("clip_gopro_64")
x = torch.from_numpy(synthetic_frames((1, 2, 3, 256, 256), 23)).cuda()
ALL0 = {"fuse": 0, "panel_gemm": 0, "dw_rows": 0, "gemm_lds": 0, "gemm_pn": 0,
        "sab_mfma": 0, "stem_mfma": 0}
for opts in ({}, ALL0):
    m = TurtleHIP(meta["opt"], dtype="bf16")
    m.load_state_dict(synth_sd({k: tuple(v.shape) for k, v in m.state_dict().items()}, meta["seed"]))
    m = m.cuda().eval()
    for k, v in opts.items():
        m.set_option(k, v)
    with torch.no_grad():
        outs = [m(x, None, None)[0].clone() for _ in range(3)]
    d = max(float((o - outs[0]).abs().max()) for o in outs[1:])
    print(opts, "max |diff| over 3 runs:", d, flush=True)
