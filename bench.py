"""Turtle GoPro deblur throughput on MI355X: restored frames/s at 1080p (bf16, 5-frame causal clips).

    python bench.py [--gpus N --steps K --warmup W] [--res 1080p|540p|256] [--dtype bf16|fp32]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 ... bench.py --gpus N

A step = one causal Turtle_t1 forward of one 1920x1080 frame (padded 1920x1088) through the HIP
library, with the history caches full (3 priming frames run before the warmup). Inputs are
synthetic frames resident in HBM; weights are the deterministic synthetic init of the GoPro
architecture (59.08 M params, random-init, no checkpoint reachable offline).
Multi-GPU: inference does not shard (a clip's frames are sequentially dependent): every rank runs
an independent clip replica ("replicas only", scaling weak); value = frames of all ranks / max
rank time. `--gpus N` without an external launcher spawns the N worker processes itself (before
any GPU call); under torch.distributed.run, WORLD_SIZE must equal N.

The JSON line also carries
* roofline: the dominant kernel launch shape (most GPU time over the warmup frames, where every
  launch is event-timed) priced with its algorithmic bytes or FLOPs per launch over its average
  duration, timed by HIP events (on the forward's stream) around exactly that shape's launches
  inside the timed region, so the events do not inflate the frame time. Bytes count each distinct
  tensor once (a fused block's residual is its own input); both the HBM and the MFMA fraction are
  given, `frac` is the binding one (arithmetic intensity vs the 312 FLOP/B ridge);
  traffic = its PMC HBM bytes per launch from profiles/pmc_traffic.json, used only when that file
  was measured on the same kernel sources (source hash), else null;
* cpu_baseline: the CPU oracle (oracle/turtle_ref.py, fp32 PyTorch CPU restatement of the
  reference, dense SAB like the reference) timed on a bounded 256x256 steady-state sample on the
  host cores, scaled to the bench resolution by the reference's own FLOP ratio F_ref
  (SURVEY.md §8(a)); host CPU model, nproc and threads stated;
* psnr_bf16_vs_fp32_db: the bf16 output vs the fp32 HIP output (itself parity-tested against the
  reference) on the same frames; psnr_delta_vs_fp32_db: |uint8 PSNR(bf16, clean) - uint8
  PSNR(fp32, clean)| on a denoising clip at the bench resolution (north star: <= 0.01 dB).
"""
from __future__ import annotations

import argparse
import shutil
import json
import math
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist
import yaml

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from turtlevsr_amd.graph import GraphedTurtle  # noqa: E402
from turtlevsr_amd.model import TurtleHIP  # noqa: E402
from turtlevsr_amd.replicas import check_world, clip_seed, launch_workers, replica_throughput  # noqa: E402
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


def f_ref(h, w):
    """The reference's FLOPs per steady-state frame (dense SAB A.v):
    5.8884e6 P1 + 2 N^2 * 101760. The CPU oracle computes the same dense graph."""
    hp, wp = (h + 31) // 32 * 32, (w + 31) // 32 * 32
    p1 = hp * wp
    n = p1 / 256
    return 5.8884e6 * p1 + 2 * n * n * 101760


def source_hash():
    """Hash of the HIP kernel sources + build script (turtlevsr_amd/build.py): ties committed PMC
    counters to the kernels they were measured on."""
    from turtlevsr_amd.build import source_hash as sh
    return sh()


def model_lib_hash():
    """Kernel-source hash compiled into the loaded libturtle_hip.so (equal to source_hash(): _lib refuses
    a stale library)."""
    from turtlevsr_amd import _lib
    return _lib.source_hash()


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def load_opt():
    with open(os.path.join(REPO, "options", "Turtle_Deblur_Gopro.yml")) as f:
        return yaml.safe_load(f)


def build_model(opt, dtype, dev, sr=False):
    m = TurtleHIP(opt, sr=sr, dtype=dtype)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    m.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(shapes, 0).items()})
    # one host->device transfer: the parameters become views of one device buffer (m.to(dev)
    # would issue one copy per parameter, ~630 copy launches in the profile)
    ps = list(m.parameters())
    flat = torch.cat([p.detach().reshape(-1) for p in ps]).to(dev)
    off = 0
    for p in ps:
        p.data = flat[off:off + p.numel()].view_as(p)
        off += p.numel()
    return m.to(dev).eval()


def denoise_clip(n, h, w, batch, dev, sigma=25.0, seed=3):
    """Smooth clean frames (x8 bilinear-upsampled noise) and noisy inputs (+ N(0, sigma/255))."""
    g = torch.Generator().manual_seed(seed)
    low = torch.rand(batch * n, 3, h // 8 + 1, w // 8 + 1, generator=g)
    clean = torch.nn.functional.interpolate(low, size=(h, w), mode="bilinear", align_corners=False)
    noisy = clean + torch.randn(clean.shape, generator=g) * (sigma / 255.0)
    return (clean.reshape(batch, n, 3, h, w).to(dev), noisy.reshape(batch, n, 3, h, w).to(dev))


def clip_frames(h, w, seed, dev, n=5, batch=1):
    clip = torch.from_numpy(synthetic_frames((batch, n, 3, h, w), seed)).to(dev)
    return [torch.stack([clip[:, max(j - 1, 0)], clip[:, j]], dim=1).contiguous() for j in range(n)]


def cpu_share_threads():
    """Host threads for the CPU baseline: the GPU box's CPU share per GPU (OMP_NUM_THREADS, 16 on the
    pool's 1-GPU boxes), capped by the cores present."""
    n = int(os.environ.get("OMP_NUM_THREADS", "16") or 16)
    return max(1, min(n, os.cpu_count() or 1))


def _grow_cache(t, n_tokens, p4):
    """A cache tensor of the small priming run, re-shaped to the bench frame size (same layout:
    FHR slots [B, heads, rows, P4], SAB slots [B, T, 1, N, d]) and filled with synthetic values."""
    if t is None:
        return None
    shape = list(t.shape)
    if t.dim() == 4:
        shape[3] = p4
    else:
        shape[3] = n_tokens
    g = torch.Generator().manual_seed(7 + t.dim() + shape[-1])
    return torch.rand(shape, generator=g) - 0.5


def cpu_baseline(opt, h, w, threads, sr=False):
    """The reference's CPU path (oracle/turtle_ref.py: fp32 torch CPU restatement, dense SAB like
    the reference) MEASURED on one steady-state frame at the bench resolution: the history caches
    are full (T = ntc frames at every cached level; their shapes come from 4 priming frames at
    64x64, re-sized to this frame, synthetic contents - the cost does not depend on them).
    Returns (seconds per frame, the oracle's output, and its input frame and caches)."""
    return oracle_steady_frame(opt, h, w, threads, sr=sr)


def oracle_steady_frame(opt, h, w, threads, sr=False, sparse_av=False):
    """One steady-state frame through the CPU oracle (see cpu_baseline): returns (seconds, out,
    frame, k caches, v caches) - the same frame and grown caches can then go through the HIP model
    (the headline size pinned to the oracle directly). sparse_av: the SAB A.v as a
    sparse product (same sum; the parity test's budget), never for the timed baseline."""
    from oracle import turtle_ref as R
    torch.set_num_threads(threads)
    m = TurtleHIP(opt)
    shapes = {k: tuple(v.shape) for k, v in m.state_dict().items()}
    sd = {k: torch.from_numpy(v) for k, v in synthetic_state_dict(shapes, 0).items()}
    small = clip_frames(64, 64, 11, "cpu")
    kc = vc = None
    with torch.no_grad():
        for j in range(4):
            _, kc, vc = R.turtle_forward(sd, opt, small[j], kc, vc)
        ho, wo = (4 * h, 4 * w) if sr else (h, w)
        hp, wp = (ho + 31) // 32 * 32, (wo + 31) // 32 * 32
        kb = [_grow_cache(t, hp * wp // 256, hp * wp // 64) for t in kc]
        vb = [_grow_cache(t, hp * wp // 256, hp * wp // 64) for t in vc]
        frame = clip_frames(h, w, 12, "cpu", n=2)[1]
        print(f"[bench] cpu baseline: one steady-state {wo}x{ho} oracle frame on {threads} threads ...",
              file=sys.stderr, flush=True)
        prev, R.SAB_SPARSE_AV = R.SAB_SPARSE_AV, sparse_av
        try:
            t0 = time.perf_counter()
            out, _, _ = R.turtle_forward(sd, opt, frame, kb, vb, sr=sr)
            dt = time.perf_counter() - t0
        finally:
            R.SAB_SPARSE_AV = prev
        return dt, out, frame, kb, vb


def hip_vs_oracle(opt, dev, out_ref, frame, kb, vb, sr=False):
    """The fp32 HIP build on the oracle frame's input and caches: PSNR (peak 1) and max |diff|."""
    m = build_model(opt, "fp32", dev, sr)
    with torch.no_grad():
        o, _, _ = m(frame.to(dev), kb, vb)
    o = o.float().cpu()
    mse = float(((o - out_ref) ** 2).mean())
    del m
    torch.cuda.empty_cache()
    return dict(psnr_db=round(10 * math.log10(1.0 / max(mse, 1e-30)), 2), max_abs=float((o - out_ref).abs().max()))


def launch_groups(dump):
    """Per kernel launch shape (the library's launch tag) of the timed region: summed ms, launches,
    algorithmic bytes and FLOPs, from the TURTLE_PROF_DUMP per-launch records."""
    groups = {}
    if not os.path.exists(dump):
        return groups
    with open(dump) as f:
        for line in f:
            parts = line.rstrip("\n").split("\t")
            if len(parts) < 5:
                continue
            g = groups.setdefault(parts[4], dict(ms=0.0, launches=0, bytes=0.0, flops=0.0))
            g["ms"] += float(parts[1]); g["launches"] += 1
            g["bytes"] += float(parts[2]); g["flops"] += float(parts[3])
    return groups


def pmc_traffic():
    """HBM bytes per launch by launch tag, from the committed rocprofv3 FETCH_SIZE / WRITE_SIZE
    passes (tools/pmc_traffic.py; FETCH_SIZE doubled for the gfx950 wide-read undercount), only
    if they were measured on the current kernel sources."""
    path = os.path.join(REPO, "profiles", "pmc_traffic.json")
    if not os.path.exists(path):
        return {}, None
    with open(path) as f:
        d = json.load(f)
    if d.get("source_hash") != source_hash():
        return {}, d.get("source")
    return d.get("per_tag", {}), d.get("source")


def roofline(wprof, wgroups, nwarm, tgroups, steps, dtype):
    """Roofline of the dominant kernel: the launch shape with the most GPU time in the profiled
    warmup frames; achieved = its algorithmic bytes (or FLOPs) per launch over its average launch
    duration, from the HIP events bracketing exactly its launches inside the timed region (on the
    forward's stream); traffic = PMC HBM bytes per launch of that shape, when profiled. The
    whole-frame class / shape breakdown comes from the warmup frames (every launch timed)."""
    if not wgroups or not tgroups:
        return None
    tag = max(tgroups, key=lambda k: tgroups[k]["ms"])
    g = tgroups[tag]
    n = max(g["launches"], 1)
    avg_s = g["ms"] * 1e-3 / n
    bpl, fpl = g["bytes"] / n, g["flops"] / n
    ridge = MFMA_PEAK[dtype] * 1e12 / (HBM_PEAK_GBS * 1e9)
    hbm_frac = bpl / avg_s / 1e9 / HBM_PEAK_GBS
    mfma_frac = fpl / avg_s / 1e12 / MFMA_PEAK[dtype]
    if fpl / max(bpl, 1.0) < ridge:
        ach = bpl / avg_s / 1e9
        roof = dict(bound="hbm", achieved=round(ach, 1), peak=HBM_PEAK_GBS, unit="GB/s", frac=round(ach / HBM_PEAK_GBS, 4))
    else:
        ach = fpl / avg_s / 1e12
        roof = dict(bound="mfma", achieved=round(ach, 2), peak=MFMA_PEAK[dtype], unit="TFLOP/s",
                    frac=round(ach / MFMA_PEAK[dtype], 4))
    per_tag, pmc_src = pmc_traffic()
    tr = per_tag.get(tag)
    roof.update(traffic=round(tr["hbm_bytes_per_launch"]) if tr else None, kernel=tag,
                hbm_frac=round(hbm_frac, 4), mfma_frac=round(mfma_frac, 4),
                arithmetic_intensity=round(fpl / max(bpl, 1.0), 1), ridge_flop_per_byte=round(ridge, 1),
                traffic_source=(f"profiles/pmc_traffic.json (rocprofv3 FETCH_SIZE x 2 + WRITE_SIZE passes, run dir {pmc_src}, "
                                f"kernel sources {source_hash()})" if tr else f"none measured on kernel sources {source_hash()}"),
                launches_per_step=g["launches"] / steps, avg_launch_us=round(avg_s * 1e6, 2),
                algorithmic_bytes_per_launch=round(bpl), algorithmic_flops_per_launch=round(fpl),
                mfma_tflops=round(fpl / avg_s / 1e12, 2), hbm_gbs=round(bpl / avg_s / 1e9, 1),
                timing="HIP events around this shape's launches only, inside the timed region",
                breakdown_from=f"{nwarm} warmup frames with every launch event-timed",
                class_ms_per_step={k: round(v["ms"] / nwarm, 3) for k, v in wprof.items()},
                top_launch_shapes_ms_per_step={k: round(wgroups[k]["ms"] / nwarm, 3)
                                               for k in sorted(wgroups, key=lambda k: -wgroups[k]["ms"])[:6]})
    return roof


def train_bench(args, world, rank, dev):
    """BASELINE config 5: Turtle GoPro training, B x 5-frame 256x256 clips per GPU, one DDP step
    (forward over the causal loop, BPTT, RCCL gradient all-reduce, AdamW) per timed step."""
    from turtlevsr_amd.train import Trainer, TurtleTrain
    opt = load_opt()
    net = TurtleTrain(opt)
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    net.load_state_dict({k: torch.from_numpy(v) for k, v in synthetic_state_dict(shapes, 0).items()})
    net = net.to(dev).train()
    # TURTLE_TRAIN_ACC=0: autograd's per-use parameter gradients instead of the in-place accumulator (A/B)
    tr = Trainer(net, amp="bf16", accumulate_grads=os.environ.get("TURTLE_TRAIN_ACC", "1") != "0")
    B = args.train_batch
    lq = torch.from_numpy(synthetic_frames((B, 5, 3, 256, 256), clip_seed(rank), name="lq")).to(dev)
    gt = (lq + 0.05 * torch.from_numpy(synthetic_frames((B, 5, 3, 256, 256), clip_seed(rank), name="gt")).to(dev)).clamp(0, 1)
    for _ in range(max(args.warmup, 1)):
        tr.train_step(lq, gt)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    loss = None
    for _ in range(args.steps):
        loss = tr.train_step(lq, gt)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    rep = replica_throughput(time.perf_counter() - t0, args.steps * B * 5, dev)
    line = {
        "metric": "training frames/sec (Turtle GoPro, 5-frame 256x256 clips, DDP)",
        "value": round(rep.value, 3), "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": round(rep.t_max / args.steps * 1e3, 3), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "bf16", "data": "synthetic clips, synthetic random-init GoPro weights",
        "config": {"workload": f"Turtle GoPro training, {B} x 5-frame 256x256 clips per GPU, BPTT through the caches, "
                               "L1, AdamW 4e-4, bf16 autocast", "global_batch": B * world, "seq_len": 5,
                   "parallelism": f"ddp{world} (RCCL)" if world > 1 else "single GPU"},
        "loss": loss,
    }
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


SCALE_RES, SCALE_BATCH = "256", 8       # north-star scaling workload: 256x256 5-frame clips, 8 per GPU


def time_frames(model, frames, steps, warmup, graph, roofline_on, world):
    """Prime the caches (3 frames), W warmup frames (every launch event-timed when roofline_on),
    then K timed frames between barriers; returns (elapsed_s, wprof, wgroups, nwarm, tgroups)."""
    state = dict(kc=None, vc=None, j=0)
    runner = GraphedTurtle(model, *frames[0].shape[:1], *frames[0].shape[-2:]) if graph else None

    def step():
        if runner is not None:
            out, state["kc"], state["vc"] = runner(frames[state["j"] % len(frames)])
        else:
            out, state["kc"], state["vc"] = model(frames[state["j"] % len(frames)], state["kc"], state["vc"])
        state["j"] += 1
        return out

    with torch.no_grad():
        for _ in range(3):           # prime the history caches (steady state: full caches)
            step()
        # warmup, profiled: every launch bracketed by HIP events -> whole-frame breakdown by kernel
        # class / launch shape, and the dominant launch shape (most GPU time)
        wdump = os.path.join("/tmp", f"turtle_bench_warm_{os.getpid()}.tsv")
        if os.path.exists(wdump):
            os.remove(wdump)
        nwarm = max(warmup, 1)
        if roofline_on:
            os.environ["TURTLE_PROF_DUMP"] = wdump
            model.profile_begin("all")
        for _ in range(nwarm):
            step()
        torch.cuda.synchronize()
        wprof = model.profile_end() if roofline_on else {}
        wgroups = launch_groups(wdump)
        dom = max(wgroups, key=lambda k: wgroups[k]["ms"]) if wgroups else None
        if world > 1:
            dist.barrier()
        # timed region: HIP events only around the dominant shape's launches (per-launch events
        # on all ~400 launches of a frame would add ~3 ms of stream bubbles to the frame time)
        dump = os.path.join("/tmp", f"turtle_bench_launches_{os.getpid()}.tsv")
        if os.path.exists(dump):
            os.remove(dump)
        if dom is not None:
            os.environ["TURTLE_PROF_DUMP"] = dump
            model.profile_begin("all", tag=dom)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        t0 = time.perf_counter()
        for _ in range(steps):
            step()
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if dom is not None:
            model.profile_end()
        os.environ.pop("TURTLE_PROF_DUMP", None)
    tgroups = launch_groups(dump)
    keep = os.environ.get("TURTLE_BENCH_DUMP")     # keep the warmup frames' per-launch records
    if keep and os.path.exists(wdump):
        shutil.copyfile(wdump, keep)
    for f in (dump, wdump):
        if os.path.exists(f):
            os.remove(f)
    return elapsed, wprof, wgroups, nwarm, tgroups


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--res", default=None, choices=list(RES),
                    help="default: 1080p on one GPU; with --gpus N > 1 the north-star scaling workload "
                         f"({SCALE_RES}x{SCALE_RES} 5-frame clips, {SCALE_BATCH} per GPU, graph replay)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--batch", type=int, default=None, help="clips per GPU restored together (B of [B,2,3,H,W])")
    ap.add_argument("--sr", action="store_true", help="TurtleSuper_t1 4x SR: LR input = res/4, output at res")
    ap.add_argument("--graph", action="store_true", help="steady-state frames replayed as captured HIP graphs (turtlevsr_amd/graph.py)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-psnr", action="store_true")
    ap.add_argument("--no-scaling-point", action="store_true",
                    help="skip the N=1 measurement of the scaling workload on the default 1-GPU line")
    ap.add_argument("--no-roofline", action="store_true", help="no per-launch HIP events in the timed region")
    ap.add_argument("--profile-all", action="store_true", help="print every kernel class's time")
    ap.add_argument("--opt", action="append", default=[], metavar="NAME=VALUE",
                    help="kernel-selection switch (turtle_set_option), repeatable; A/B runs only")
    ap.add_argument("--train", action="store_true",
                    help="config 5: one DDP training step per `step` (8 x 5-frame 256x256 clips per GPU, bf16 autocast, AdamW)")
    ap.add_argument("--train-batch", type=int, default=8)
    args = ap.parse_args(argv)
    default_line, _ = resolve_workload(args)
    return args, default_line


def resolve_workload(args):
    """Workload of a run: with no --res / --batch, one GPU measures the headline configuration
    (1080p, B = 1, eager: BASELINE.json's metric) and `--gpus N > 1` the north-star scaling
    workload (256x256 5-frame clips, SCALE_BATCH per GPU, graph replay), which the default 1-GPU
    line also measures once as `scaling_workload_n1`. Returns (default 1-GPU line?, scaling run?)."""
    default_line = args.res is None and args.batch is None and not args.sr and not args.train and not args.graph
    scaling_run = args.res is None and args.gpus > 1 and not args.train and not args.sr
    if args.res is None:
        args.res = SCALE_RES if scaling_run else "1080p"
    if args.batch is None:
        args.batch = SCALE_BATCH if scaling_run else 1
    if scaling_run:
        args.graph = True
    if args.graph:
        args.no_roofline = True      # per-launch profiling events cannot live inside a captured graph
    return default_line and args.gpus == 1, scaling_run


def main():
    args, default_line = parse_args()

    # one process per GPU: spawn the workers here, before this process touches the GPU, unless an
    # external launcher (torch.distributed.run) already did; its WORLD_SIZE must match --gpus
    if check_world(args.gpus) is None and args.gpus > 1:
        sys.exit(launch_workers(args.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    if args.train:
        return train_bench(args, world, rank, dev)
    h, w = RES[args.res]
    opt = load_opt()

    model = build_model(opt, args.dtype, dev, args.sr)
    for kv in args.opt:
        name, value = kv.split("=", 1)
        model.set_option(name, int(value))
    if args.sr:
        if h % 4 or w % 4:
            raise SystemExit(f"--sr needs an output size divisible by 4, got {w}x{h}")
        frames = clip_frames(h // 4, w // 4, clip_seed(rank), dev, batch=args.batch)
    else:
        frames = clip_frames(h, w, clip_seed(rank), dev, batch=args.batch)
    elapsed, wprof, wgroups, nwarm, tgroups = time_frames(model, frames, args.steps, args.warmup, args.graph,
                                                          not args.no_roofline, world)
    rep = replica_throughput(elapsed, args.steps * args.batch, dev)
    tmax, fps = rep.t_max, rep.value
    roof = roofline(wprof, wgroups, nwarm, tgroups, args.steps, args.dtype)

    psnr = dpsnr = None
    if not args.no_psnr and rank == 0 and args.dtype == "bf16":
        from turtlevsr_amd.harness import calc_PSNR, tensor2img
        ref = build_model(opt, "fp32", dev, args.sr)
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
            # north-star PSNR delta: a denoising clip (smooth clean frames + N(0, 25/255)) through the
            # fp32 and bf16 builds, uint8 PSNR vs the clean frames (inference.py:52-61, 324-325)
            clean, noisy = denoise_clip(4, h // 4 if args.sr else h, w // 4 if args.sr else w, args.batch, dev)
            kr = vr = kb = vb = None
            deltas = []
            for jj in range(4):
                x = torch.stack([noisy[:, max(jj - 1, 0)], noisy[:, jj]], dim=1).contiguous()
                o32, kr, vr = ref(x, kr, vr)
                o16, kb, vb = model(x, kb, vb)
                if args.sr:
                    gt = torch.nn.functional.interpolate(clean[:, jj], scale_factor=4, mode="bilinear", align_corners=False)
                else:
                    gt = clean[:, jj]
                p32 = calc_PSNR(tensor2img(o32[0]), tensor2img(gt[0]))
                p16 = calc_PSNR(tensor2img(o16[0]), tensor2img(gt[0]))
                deltas.append(abs(p16 - p32))
            dpsnr = round(max(deltas), 5)
        del ref

    # the scaling workload at N = 1 (the default line only): the point the driver's N > 1 runs of
    # `--gpus N` (which default to that workload) are compared with
    scale_pt = None
    if default_line and world == 1 and rank == 0 and not args.no_scaling_point:
        del model
        torch.cuda.empty_cache()
        sh, sw = RES[SCALE_RES]
        sm = build_model(opt, args.dtype, dev)
        sframes = clip_frames(sh, sw, clip_seed(rank), dev, batch=SCALE_BATCH)
        s_el, *_ = time_frames(sm, sframes, max(args.steps, 10), 3, True, False, 1)
        scale_pt = dict(value=round(max(args.steps, 10) * SCALE_BATCH / s_el, 3), unit="frames/s", n_gpus=1,
                        workload=f"Turtle_t1 GoPro deblur, {sw}x{sh} causal 5-frame clips, B={SCALE_BATCH} per GPU, "
                                 "caches full, HIP graph replay (the `--gpus N > 1` default workload)")
        del sm

    cpu = parity = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        threads = cpu_share_threads()
        dt, out_ref, oframe, okb, ovb = cpu_baseline(opt, h // 4 if args.sr else h, w // 4 if args.sr else w, threads,
                                                     sr=args.sr)
        pin = hip_vs_oracle(opt, dev, out_ref, oframe, okb, ovb, sr=args.sr)
        cpu = dict(value=round(1.0 / dt, 6), unit="frames/s", cores=threads, kind="port", measured=True,
                   s_per_frame=round(dt, 2), cpu_model=cpu_model(), nproc=os.cpu_count(),
                   torch_threads=torch.get_num_threads(),
                   sample=f"oracle/turtle_ref.py fp32 (dense SAB, as the reference), ONE steady-state {w}x{h} frame "
                          f"(history caches full: T = ntc at every cached level), B=1, timed on {threads} host threads "
                          f"(the box's CPU share per GPU): {dt:.1f} s/frame; not extrapolated")
        # the same frame, input and grown caches through the fp32 HIP build
        parity = dict(psnr_fp32_vs_oracle_db=pin["psnr_db"], max_abs=pin["max_abs"],
                      frame=f"the cpu_baseline frame: steady-state {oframe.shape[-1]}x{oframe.shape[-2]}, caches full, fp32 HIP vs the oracle")

    line = {
        "metric": "restored frames/sec @1080p (1/2/4/8 GPU) + PSNR delta vs ref"
        if args.res == "1080p" and not args.sr and args.batch == 1
        else f"restored frames/sec @{args.res}" + (" (4x SR output)" if args.sr else "") + (f" B={args.batch}" if args.batch > 1 else ""),
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
        "config": {"workload": (f"TurtleSuper_t1 GoPro-arch 4x SR, {w // 4}x{h // 4} -> {w}x{h}" if args.sr
                                else f"Turtle_t1 GoPro deblur, {w}x{h}") + f", causal 5-frame clip, B={args.batch} per GPU, caches full",
                   "model": "Turtle_t1 (GoPro arch, 59.08M params)", "global_batch": world * args.batch, "seq_len": 5,
                   "parallelism": f"replicas x{world}",
                   "execution": "HIP graph replay (2 captured graphs, ping-pong caches)" if args.graph else "eager launches"},
        "roofline": roof,
        "cpu_baseline": cpu,
        "psnr_bf16_vs_fp32_db": psnr,
        "psnr_delta_vs_fp32_db": dpsnr,
        "parity_fp32_vs_oracle": parity,
        "lib_source_hash": model_lib_hash(),
        "alg_tflops": round(f_alg(h, w) * fps / 1e12, 2),
    }
    if scale_pt is not None:
        line["scaling_workload_n1"] = scale_pt
    if rank == 0:
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
