"""Golden vectors for the t0 network ("Turtle", basicsr/models/archs/turtle_arch.py): SURVEY.md
§8(f) rank 4. Same procedure as gen_golden.py (reference arch loaded by file path in the build
container only, deterministic synthetic weights, data-only .npz outputs):

    python tests/golden/gen_golden_t0.py

* ``clip_tiny_t0.npz``  - tiny widths, 5-frame 64x64 causal clip: every output, the last frame's
                          caches in full (t0's k cache is the dilated ws*ws*c token of k);
* ``clip_gopro_t0.npz`` - GoPro widths, 3-frame 64x64 clip: outputs + cache checksums;
* ``block_sab_t0.npz``  - the t0 StateAlignBlock alone (c=32, ws=8, 2-frame cache).
The option dicts carry ``model: Turtle_arch`` (Turtle_Derain.yml / Turtle_Desnow.yml select it)."""
from __future__ import annotations

import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from gen_golden import arch_opt, fill, gopro_opt, load_by_path, run_clip, save, tiny_opt  # noqa: E402
from turtlevsr_amd.synthetic import synthetic_frames, synthetic_state_dict  # noqa: E402


def main():
    torch.set_num_threads(8)
    t0 = load_by_path("basicsr/models/archs/turtle_arch.py", "ref_turtle_t0")
    for name, opt, shape, full, seed in [
        ("clip_tiny_t0", tiny_opt(model="Turtle_arch"), (1, 5, 3, 64, 64), True, 21),
        ("clip_gopro_t0", dict(gopro_opt(), model="Turtle_arch"), (1, 3, 3, 64, 64), False, 22),
    ]:
        torch.manual_seed(0)
        model = t0.make_model(opt).eval()
        fill(model, seed)
        clip = synthetic_frames(shape, seed, name="frames")
        rec = run_clip(model, clip, full)
        rec["clip"] = clip
        meta_opt = arch_opt(opt)
        meta_opt["model"] = "Turtle_arch"
        save(name, rec, dict(opt=meta_opt, seed=seed, sr=False, shape=list(shape)))

    rng_seed = 101
    m = t0.StateAlignBlock(32, 1, False, 2, Scale_patchsize=4).eval()
    shapes = {"blk." + k: tuple(v.shape) for k, v in m.state_dict().items() if v is not None}
    sd = synthetic_state_dict(shapes, rng_seed)
    m.load_state_dict({k[4:]: torch.from_numpy(v) for k, v in sd.items()}, strict=False)

    def frames(shp, nm):
        return torch.from_numpy(synthetic_frames(shp, rng_seed, name=nm) * 2.0 - 1.0)

    with torch.no_grad():
        x = frames((1, 32, 32, 24), "sab0_x")                       # 4x3 = 12 tokens of 8*8*32
        kc = torch.nn.functional.normalize(frames((1, 2, 1, 12, 8 * 8 * 32), "sab0_kc"), dim=-1)
        vc = frames((1, 2, 1, 12, 8 * 8 * 32), "sab0_vc")
        y, k, v = m(x, kc, vc)
        y0, k0, v0 = m(x)
    save("block_sab_t0", {"x": x.numpy(), "kc": kc.numpy(), "vc": vc.numpy(), "y": y.numpy(), "k": k.numpy(),
                          "v": v.numpy(), "y0": y0.numpy(), "k0": k0.numpy(), "v0": v0.numpy()},
         dict(dim=32, ws=8, ntc=2, seed=rng_seed))


if __name__ == "__main__":
    main()
