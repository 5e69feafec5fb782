"""Where does the bf16 - fp32 uint8-PSNR delta at 1080p come from?

    python tools/psnr_probe.py [--res 1080p] [--seeds 3,4] [--opt NAME=VALUE ...]

Runs bench.py's denoising clip (smooth clean frames + N(0, 25/255)) through the fp32 build, the
bf16 build and the fp32 build with bf16-rounded weights, and prints per frame: the uint8 PSNR
delta, the float PSNR delta (no uint8 rounding), and the error decomposition
dMSE = 2 E[e (o32 - clean)] + E[e^2] with e = o16 - o32, plus the scale coefficient
delta = E[e r] / E[r^2] of e on the fp32 network residual r = o32 - noisy.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import bench  # noqa: E402
from turtlevsr_amd.harness import calc_PSNR, tensor2img  # noqa: E402


def run(model, noisy, n):
    kc = vc = None
    outs = []
    with torch.no_grad():
        for j in range(n):
            x = torch.stack([noisy[:, max(j - 1, 0)], noisy[:, j]], dim=1).contiguous()
            o, kc, vc = model(x, kc, vc)
            outs.append(o.float().clone())
    return outs


def weight_class(k, v):
    if k.endswith("temperature") or k.endswith("beta") or k.endswith("gamma"):
        return "scalar"
    if ".norm" in k:
        return "ln"
    if k.endswith(".bias"):
        return "bias"
    if v.dim() == 4 and v.shape[1] == 1 and v.shape[0] > 1:
        return "dw"
    if v.dim() == 4 and v.shape[2] == 1:
        return "pw"
    return "dense"


def fpsnr(a, b):
    return float(10 * np.log10(1.0 / float(((a.clamp(0, 1) - b) ** 2).mean())))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--res", default="1080p")
    ap.add_argument("--seeds", default="3")
    ap.add_argument("--frames", type=int, default=4)
    ap.add_argument("--opt", action="append", default=[])
    ap.add_argument("--wround", action="store_true", help="also the fp32 build with bf16-rounded weights")
    ap.add_argument("--subsets", action="store_true",
                    help="fp32 builds with one weight class rounded to bf16 at a time (pw, dw, dense, ln, scalar, bias)")
    ap.add_argument("--by-module", action="store_true", help="with --subsets: pw / dense weights of one top-level module at a time")
    args = ap.parse_args()
    h, w = bench.RES[args.res]
    dev = torch.device("cuda", 0)
    opt = bench.load_opt()
    m32 = bench.build_model(opt, "fp32", dev)
    m16 = bench.build_model(opt, "bf16", dev)
    for kv in args.opt:
        k, v = kv.split("=", 1)
        m16.set_option(k, int(v))
    mw = None
    if args.wround:
        mw = bench.build_model(opt, "fp32", dev)
        mw.load_state_dict({k: v.to(torch.bfloat16).float() for k, v in mw.state_dict().items()})
    if args.subsets:
        seed = int(args.seeds.split(",")[0])
        clean, noisy = bench.denoise_clip(args.frames, h, w, 1, dev, seed=seed)
        o32 = run(m32, noisy, args.frames)
        del m16
        torch.cuda.empty_cache()
        classes = ("pw", "dw", "dense", "ln", "scalar", "bias")
        if args.by_module:
            mods = sorted({k.split(".")[0] for k in m32.state_dict()})
            classes = [f"{c}:{m}" for c in ("pw", "dense") for m in mods]
        for cls in classes:
            mc = bench.build_model(opt, "fp32", dev)
            sd = mc.state_dict()
            n = 0
            new = {}
            for k, v in sd.items():
                if weight_class(k, v) == cls or (":" in cls and cls == weight_class(k, v) + ":" + k.split(".")[0]):
                    new[k] = v.to(torch.bfloat16).float()
                    n += v.numel()
                else:
                    new[k] = v
            if n == 0:
                del mc
                continue
            mc.load_state_dict(new)
            oc = run(mc, noisy, args.frames)
            for j in range(args.frames):
                g8 = tensor2img(clean[0, j])
                p32 = calc_PSNR(tensor2img(o32[j][0]), g8)
                r = o32[j] - noisy[:, j]
                ec = oc[j] - o32[j]
                print(json.dumps(dict(cls=cls, numel=n, frame=j, d_u8=round(calc_PSNR(tensor2img(oc[j][0]), g8) - p32, 5),
                                      scale=float((ec * r).mean() / r.pow(2).mean()),
                                      psnr_vs_32=round(float(10 * np.log10(1.0 / float(ec.pow(2).mean()))), 2))), flush=True)
            del mc
            torch.cuda.empty_cache()
        return
    for seed in [int(s) for s in args.seeds.split(",")]:
        clean, noisy = bench.denoise_clip(args.frames, h, w, 1, dev, seed=seed)
        o32 = run(m32, noisy, args.frames)
        o16 = run(m16, noisy, args.frames)
        ow = run(mw, noisy, args.frames) if mw is not None else None
        for j in range(args.frames):
            gt = clean[:, j]
            g8 = tensor2img(gt[0])
            p32 = calc_PSNR(tensor2img(o32[j][0]), g8)
            p16 = calc_PSNR(tensor2img(o16[j][0]), g8)
            e = o16[j] - o32[j]
            err = o32[j].clamp(0, 1) - gt
            r = o32[j] - noisy[:, j]
            rec = dict(seed=seed, frame=j, p32=round(p32, 5), d_u8=round(p16 - p32, 5),
                       d_float=round(fpsnr(o16[j], gt) - fpsnr(o32[j], gt), 5),
                       mse32=float((err ** 2).mean()), e_rms=float(e.pow(2).mean().sqrt()), e_mean=float(e.mean()),
                       cross=float((e * err).mean()), r_rms=float(r.pow(2).mean().sqrt()),
                       scale=float((e * r).mean() / r.pow(2).mean()),
                       psnr_16_vs_32=round(float(10 * np.log10(1.0 / float(e.pow(2).mean()))), 2))
            if ow is not None:
                rec["d_u8_wround"] = round(calc_PSNR(tensor2img(ow[j][0]), g8) - p32, 5)
                ew = ow[j] - o32[j]
                rec["scale_wround"] = float((ew * r).mean() / r.pow(2).mean())
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
