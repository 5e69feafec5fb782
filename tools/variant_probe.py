"""bf16 PSNR vs the fp32 build of kernel-switch variants on the synthetic 128x128 GoPro-width clip
of tests/test_hip_parity.py::test_kernel_variants_agree (which switch breaks a variant?).
    python tools/variant_probe.py "split_out=0" "split_out=1" ...   (or VPROBE="a=1;b=0 c=1")"""
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
from golden_io import load, synth_sd  # noqa: E402
from turtlevsr_amd.model import TurtleHIP  # noqa: E402
from turtlevsr_amd.synthetic import synthetic_frames  # noqa: E402

BASE = {"fuse": 0, "fused2": 0, "panel_gemm": 0, "dw_rows": 0, "gemm_lds": 0, "gemm_pn": 0,
        "sab_mfma": 0, "stem_mfma": 0, "gemm_ar": 0, "gemm_kt": 0, "dwgemm": 0,
        "dwgemm_min_blocks": 0, "ffn": 0, "down_tile": 0}


def run(meta, dtype, opts, clip):
    m = TurtleHIP(meta["opt"], sr=meta["sr"], dtype=dtype)
    m.load_state_dict(synth_sd({k: tuple(t.shape) for k, t in m.state_dict().items()}, meta["seed"]))
    m = m.cuda().eval()
    for k, v in opts.items():
        m.set_option(k, v)
    x = torch.from_numpy(clip).cuda()
    kc = vc = None
    outs = []
    with torch.no_grad():
        for j in range(x.shape[1]):
            o, kc, vc = m(torch.stack([x[:, max(j - 1, 0)], x[:, j]], 1), kc, vc)
            outs.append(o.float().cpu().numpy())
    return outs


def psnr(a, b):
    return 10 * np.log10(1.0 / max(float(np.mean((a - b) ** 2)), 1e-20))


_, meta = load("clip_gopro_64")
clip = synthetic_frames((1, 3, 3, 128, 128), 11)
ref = run(meta, "fp32", BASE, clip)
for spec in sys.argv[1:] or os.environ.get("VPROBE", ";split_out=0").split(";"):
    opts = dict(BASE)
    for kv in spec.split():
        k, v = kv.split("=")
        opts[k] = int(v)
    o = run(meta, "bf16", opts, clip)
    print(f"[{spec}] bf16 vs fp32 dB per frame: {[round(psnr(a, r), 2) for a, r in zip(o, ref)]}", flush=True)
