"""Turtle GoPro deblur throughput on MI355X: restored frames/s at 1080p (bf16, 5-frame causal clips).

    python bench.py [--gpus N --steps K --warmup W] [--res 1080p|540p|256] [--dtype bf16|fp32]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

A step = one causal Turtle_t1 forward of one 1920x1080 frame (padded 1920x1088) through the HIP
library, with the history caches full (3 priming frames run before the warmup). Inputs are
synthetic frames resident in HBM; weights are the deterministic synthetic init of the GoPro
architecture (59.08 M params, random-init, no checkpoint reachable offline).
Multi-GPU: inference does not shard (a clip's frames are sequentially dependent): every rank runs
an independent clip replica ("replicas only", scaling weak); value = frames of all ranks / max
rank time.

The JSON line also carries
* roofline: the dominant kernel class (most GPU time in the timed region, measured with HIP
  events on the forward's stream) priced with its algorithmic bytes or FLOPs per launch;
* cpu_baseline: the CPU oracle (oracle/turtle_ref.py, fp32 PyTorch CPU restatement of the
  reference) on a bounded 256x256 steady-state sample, scaled to 1080p frames/s by the
  algorithmic FLOP ratio;
* psnr_bf16_vs_fp32_db: the bf16 output vs the fp32 HIP output (itself parity-tested against the
  reference) on the same 1080p frames.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist
import yaml

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from turtlevsr_amd.model import TurtleHIP  # noqa: E402
from turtlevsr_amd.synthetic import synthetic_frames, synthetic_state_dict  # noqa: E402

RES = {"1080p": (1080, 1920), "540p": (540, 960), "256": (256, 256), "128": (128, 128)}
HBM_PEAK_GBS = 8000.0          # MI355X_MICROARCH.md: 8 TB/s spec
MFMA_PEAK = {"bf16": 2500.0, "fp32": 157.3}   # dense TFLOP/s


def f_alg(h, w):
    """Algorithmic FLOPs per steady-state frame (sparse SAB)."""
    hp, wp = (h + 31) // 32 * 32, (w + 31) // 32 * 32
    p1 = hp * wp
    n = p1 / 256
    return 5.8884e6 * p1 + 6912 * n * n + 9.0440e6 * n


def load_opt():
    with open(os.path.join(REPO, "options", "Turtle_Deblur_Gopro.yml")) as f:
        return yaml.safe_load(f)


def build_model(opt, dtype, dev):
    m = TurtleHIP(opt, dtype=dtype)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(shapes, 0).items()})
    return m.to(dev).eval()


def clip_frames(h, w, seed, dev, n=5):
    clip = torch.from_numpy(synthetic_frames((1, n, 3, h, w), seed)).to(dev)
    return [torch.stack([clip[:, max(j - 1, 0)], clip[:, j]], dim=1).contiguous() for j in range(n)]


def cpu_baseline(opt, threads):
    """Oracle fp32 on a 256x256 steady-state frame (3 priming frames untimed, 2 timed)."""
    from oracle import turtle_ref as R
    torch.set_num_threads(threads)
    m = TurtleHIP(opt)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    sd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(shapes, 0).items()}
    frames = clip_frames(256, 256, 11, "cpu")
    kc = vc = None
    for j in range(3):
        _, kc, vc = R.turtle_forward(sd, opt, frames[j], kc, vc)
    t0 = time.perf_counter()
    for j in range(3, 5):
        _, kc, vc = R.turtle_forward(sd, opt, frames[j], kc, vc)
    dt = (time.perf_counter() - t0) / 2
    return dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--res", default="1080p", choices=list(RES))
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-psnr", action="store_true")
    ap.add_argument("--profile-all", action="store_true", help="print every kernel class's time")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    h, w = RES[args.res]
    opt = load_opt()

    model = build_model(opt, args.dtype, dev)
    frames = clip_frames(h, w, 100 + rank, dev)
    kc = vc = None
    j = 0

    def step():
        nonlocal kc, vc, j
        out, kc, vc = model(frames[j % len(frames)], kc, vc)
        j += 1
        return out

    with torch.no_grad():
        for _ in range(3):           # prime the history caches (steady state: full caches)
            step()
        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        model.profile_begin("all")
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            out = step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        prof = model.profile_end()
    t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    tmax = float(t.item())
    frames_total = args.steps * world
    fps = frames_total / tmax

    # dominant kernel class in the timed region
    dom = max(prof, key=lambda k: prof[k]["ms"])
    pd = prof[dom]
    per_launch_ms = pd["ms"] / max(pd["launches"], 1)
    gbs = pd["bytes"] / (pd["ms"] * 1e-3) / 1e9 if pd["ms"] > 0 else 0.0
    tfs = pd["flops"] / (pd["ms"] * 1e-3) / 1e12 if pd["ms"] > 0 else 0.0
    # bound: arithmetic intensity of the class vs the MFMA ridge
    ridge = MFMA_PEAK[args.dtype] * 1e12 / (HBM_PEAK_GBS * 1e9)
    ai = pd["flops"] / max(pd["bytes"], 1.0)
    if ai < ridge:
        roof = dict(bound="hbm", achieved=round(gbs, 1), peak=HBM_PEAK_GBS, unit="GB/s", frac=round(gbs / HBM_PEAK_GBS, 4))
    else:
        roof = dict(bound="mfma", achieved=round(tfs, 2), peak=MFMA_PEAK[args.dtype], unit="TFLOP/s",
                    frac=round(tfs / MFMA_PEAK[args.dtype], 4))
    roof.update(kernel=dom, launches_per_step=pd["launches"] / args.steps, avg_launch_us=round(per_launch_ms * 1e3, 2),
                algorithmic_bytes_per_launch=pd["bytes"] / max(pd["launches"], 1),
                algorithmic_flops_per_launch=pd["flops"] / max(pd["launches"], 1), traffic=None,
                class_ms_per_step={k: round(v["ms"] / args.steps, 3) for k, v in prof.items()})

    psnr = None
    if not args.no_psnr and rank == 0 and args.dtype == "bf16":
        ref = build_model(opt, "fp32", dev)
        kr = vr = None
        kb = vb = None
        vals = []
        with torch.no_grad():
            for jj in range(4):
                o32, kr, vr = ref(frames[jj], kr, vr)
                o16, kb, vb = model(frames[jj], kb, vb)
                mse = float(((o32 - o16) ** 2).mean())
                vals.append(10 * np.log10(1.0 / max(mse, 1e-20)))
        psnr = round(min(vals), 2)
        del ref

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = min(16, os.cpu_count() or 1)
        dt = cpu_baseline(opt, threads)
        scale = f_alg(256, 256) / f_alg(h, w)
        cpu = dict(value=round(scale / dt, 6), unit="frames/s", cores=threads, kind="port",
                   sample=f"oracle/turtle_ref.py fp32 on 2 steady-state 256x256 GoPro frames ({dt:.2f} s/frame, "
                          f"{threads} threads), scaled to {args.res} by F_alg ratio {scale:.5f}")

    line = {
        "metric": "restored frames/sec @1080p (1/2/4/8 GPU) + PSNR delta vs ref" if args.res == "1080p"
        else f"restored frames/sec @{args.res}",
        "value": round(fps, 3),
        "unit": "frames/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(tmax / args.steps * 1e3, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": args.dtype,
        "data": "synthetic frames (uniform [0,1)), synthetic random-init GoPro weights",
        "config": {"workload": f"Turtle_t1 GoPro deblur, causal 5-frame clip, {w}x{h}, B=1, caches full",
                   "model": "Turtle_t1 (GoPro arch, 59.08M params)", "global_batch": world, "seq_len": 5,
                   "parallelism": f"replicas x{world}"},
        "roofline": roof,
        "cpu_baseline": cpu,
        "psnr_bf16_vs_fp32_db": psnr,
        "alg_tflops": round(f_alg(h, w) * fps / 1e12, 2),
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
