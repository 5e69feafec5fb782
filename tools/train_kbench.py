"""Per-launch times of the training step's elementwise / reduction kernels at the config-5 level
shapes (8 x 256^2 clips: level 1..latent), bf16, through the C ABI (GPU box):

    python tools/train_kbench.py            # TURTLE_TRAIN_ABL=1: without the end-of-block global atomics

Prints us per launch and the algorithmic GB/s (each tensor read / written once)."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from turtlevsr_amd import train_ops as T  # noqa: E402

dev = torch.device("cuda", 0)
L = T.lib()
st = C.c_void_p(torch.cuda.current_stream().cuda_stream)
p = lambda t: C.c_void_p(t.data_ptr()) if t is not None else None


def timeit(fn, it=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / it


SHAPES = [("L1", 8 * 256 * 256, 64), ("L2", 8 * 128 * 128, 128), ("L3", 8 * 64 * 64, 256), ("lat", 8 * 32 * 32, 512)]
print(f"TURTLE_TRAIN_ABL={os.environ.get('TURTLE_TRAIN_ABL', '0')} TURTLE_TRAIN_TUNE={os.environ.get('TURTLE_TRAIN_TUNE', '')}")
# weight-gradient reduction GEMMs dW[N][K] = dy^T x over P pixels (config-5 shapes: GatedFFN project_in /
# project_out, qkv, 64 x 64) - algorithmic bytes = dy + x once (the partials are overhead)
# forward / input-gradient GEMMs y[P][N] = x[P][K] W^T (the inference GEMM family; the dgrad shapes have
# the wide K): algorithmic bytes = x + W + y once
for P, K, N in ((524288, 64, 320), (524288, 320, 64), (524288, 160, 64), (524288, 64, 160), (131072, 128, 640),
                (131072, 640, 128), (131072, 320, 128), (32768, 256, 1280), (32768, 1280, 256), (8192, 512, 2560),
                (8192, 2560, 512)):
    x = torch.randn(P, K, device=dev).to(torch.bfloat16)
    w = (0.05 * torch.randn(N, K, device=dev)).to(torch.bfloat16)
    y = torch.empty(P, N, device=dev, dtype=torch.bfloat16)
    fn = lambda: L.turtle_train_gemm(p(x), K, p(w), 0, 0, None, None, 0, p(y), N, P, K, N, 1, st)
    assert fn() == 0
    us = timeit(fn)
    mb = (P * (K + N) + N * K) * 2 / 1e6
    print(f"gemm  P={P:7d} K={K:5d} N={N:4d} {us:8.1f} us  {mb / us:6.2f} TB/s  {2 * P * K * N / us / 1e6:7.1f} TF/s")
for P, N, K in ((524288, 320, 64), (524288, 64, 160), (524288, 192, 64), (524288, 64, 64), (131072, 640, 128),
                (131072, 128, 320), (32768, 1280, 256), (8192, 2560, 512)):
    a = torch.randn(P, N, device=dev).to(torch.bfloat16)
    b_ = torch.randn(P, K, device=dev).to(torch.bfloat16)
    c = torch.zeros(N, K, device=dev)
    nws = int(L.turtle_train_rgemm_workspace(P, N, K, 0))
    ws = torch.empty(max(nws, 16), dtype=torch.uint8, device=dev)
    fn = lambda: L.turtle_train_rgemm(p(a), N, p(b_), K, p(c), P, N, K, 0, 1, 1, p(ws), ws.numel(), st)
    us = timeit(fn)
    mb = P * (N + K) * 2 / 1e6
    print(f"rgemm P={P:7d} N={N:5d} K={K:4d} {us:8.1f} us  {mb / us:6.2f} TB/s  partials {nws / 1e6:7.1f} MB")
for name, P, Cc in SHAPES:
    x = torch.randn(P, Cc, device=dev).to(torch.bfloat16)
    dy = torch.randn(P, Cc, device=dev).to(torch.bfloat16)
    dr = torch.randn(P, Cc, device=dev).to(torch.bfloat16)
    y = torch.empty_like(x)
    dx = torch.empty_like(x)
    w = torch.ones(Cc, device=dev)
    b = torch.zeros(Cc, device=dev)
    mu = torch.empty(P, device=dev)
    rs = torch.empty(P, device=dev)
    dw = torch.zeros(Cc, device=dev)
    db = torch.zeros(Cc, device=dev)
    mb = P * Cc * 2 / 1e6
    f_ln = lambda: L.turtle_train_ln_fwd(p(x), Cc, p(w), p(b), p(y), Cc, p(mu), p(rs), P, Cc, 0, 1, st)
    f_lb = lambda: L.turtle_train_ln_bwd(p(x), Cc, p(w), p(mu), p(rs), p(dy), Cc, p(dx), Cc, p(dr), Cc, p(dw), p(db), P, Cc, 0, 1, st)
    f_lb0 = lambda: L.turtle_train_ln_bwd(p(x), Cc, p(w), p(mu), p(rs), p(dy), Cc, p(dx), Cc, None, 0, p(dw), p(db), P, Cc, 0, 1, st)
    f_cs = lambda: L.turtle_train_colsum(p(dy), Cc, p(db), P, Cc, 1, st)
    H = int((P // 8) ** 0.5)
    dw9 = torch.zeros(9 * Cc, device=dev)
    f_dw = lambda: L.turtle_train_dw3x3_wgrad(p(x), Cc, p(dy), Cc, p(dw9), p(db), 8, Cc, H, H, 1, st)
    w9 = torch.ones(9, Cc, device=dev)
    f_df = lambda: L.turtle_train_dw3x3_fwd(p(x), Cc, p(w9), None, p(y), Cc, 8, Cc, H, H, 0, 1, st)
    h = 5 * Cc // 2                                  # the GatedFFN hidden width (ffn_expansion_factor 2.5)
    xg = torch.randn(P, 2 * h, device=dev).to(torch.bfloat16)
    gg = torch.randn(P, h, device=dev).to(torch.bfloat16)
    yg = torch.empty(P, h, device=dev, dtype=torch.bfloat16)
    dxg = torch.empty(P, 2 * h, device=dev, dtype=torch.bfloat16)
    f_gf = lambda: L.turtle_train_gate_fwd(p(xg), 2 * h, p(yg), h, P, h, 1, st)
    f_gb = lambda: L.turtle_train_gate_bwd(p(xg), 2 * h, p(gg), h, p(dxg), 2 * h, P, h, 1, st)
    mbh = P * h * 2 / 1e6
    for tag, fn, gb in (("gate_fwd", f_gf, 3 * mbh), ("gate_bwd", f_gb, 5 * mbh), ("ln_fwd", f_ln, 2 * mb), ("ln_bwd+res", f_lb, 4 * mb), ("ln_bwd", f_lb0, 3 * mb), ("colsum", f_cs, mb),
                        ("dw_wgrad", f_dw, 2 * mb), ("dw_fwd", f_df, 2 * mb)):
        us = timeit(fn)
        print(f"{name:4s} P={P:7d} C={Cc:4d} {tag:11s} {us:8.1f} us  {gb / us:6.2f} TB/s")
