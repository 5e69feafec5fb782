"""bf16 PSNR of a golden clip under kernel-switch variants (which switch breaks bf16 parity?).
    python tools/bf16_isolate.py [clip_gopro_64] ["split_out=0" "ffn=0" ...]"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from golden_io import clip_input, load, synth_sd  # noqa: E402
from turtlevsr_amd.model import TurtleHIP  # noqa: E402

name = sys.argv[1] if len(sys.argv) > 1 else "clip_gopro_64"
variants = sys.argv[2:] or ["", "split_out=0"]
g, meta = load(name)
clip = torch.from_numpy(clip_input(g, meta)).cuda()
for v in variants:
    m = TurtleHIP(meta["opt"], sr=meta["sr"], dtype="bf16")
    m.load_state_dict(synth_sd({k: tuple(t.shape) for k, t in m.state_dict().items()}, meta["seed"]))
    m = m.cuda().eval()
    for kv in v.split():
        k, val = kv.split("=")
        m.set_option(k, int(val))
    kc = vc = None
    vals = []
    with torch.no_grad():
        for j in range(clip.shape[1]):
            o, kc, vc = m(torch.stack([clip[:, max(j - 1, 0)], clip[:, j]], 1), kc, vc)
            if f"out{j}" in g:
                mse = float(np.mean((o.float().cpu().numpy() - g[f"out{j}"]) ** 2))
                vals.append(round(10 * np.log10(1 / mse), 2))
    print(f"[{v}] bf16 PSNR per frame: {vals}", flush=True)
