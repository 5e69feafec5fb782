"""Time the training graph's convolution shapes (fwd + bwd, bf16 autocast) in NCHW vs channels_last,
to see which ones fall onto MIOpen's naive kernels. GPU box only: python tools/conv_probe.py"""
import time

import torch
import torch.nn.functional as F

dev = "cuda"
B = 8
shapes = [  # name, cin, cout, k, stride, pad, groups, H
    ("1x1 64->320 L1", 64, 320, 1, 1, 0, 1, 256),
    ("1x1 256->1280 L3", 256, 1280, 1, 1, 0, 1, 64),
    ("win16 dec1", 128, 128, 16, 16, 1, 128, 256),
    ("win8 dec2", 256, 256, 8, 8, 1, 256, 128),
    ("win4 dec3", 512, 512, 4, 4, 1, 512, 64),
    ("3x3 stem 3->64", 3, 64, 3, 1, 1, 1, 256),
    ("3x3 ending 64->3", 64, 3, 3, 1, 1, 1, 256),
    ("3x3 down 64->32", 64, 32, 3, 1, 1, 1, 256),
    ("3x3 up 512->1024", 512, 1024, 3, 1, 1, 1, 32),
    ("3x3 up 128->256", 128, 256, 3, 1, 1, 1, 128),
]


def run(name, cin, cout, k, s, p, g, H, cl):
    x = torch.randn(B, cin, H, H, device=dev)
    w = torch.randn(cout, cin // g, k, k, device=dev, requires_grad=True)
    if cl:
        x = x.to(memory_format=torch.channels_last)
    x.requires_grad_()
    def step():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = F.conv2d(x, w, None, s, p, 1, g)
        y.float().sum().backward()
    for _ in range(2):
        step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / 5 * 1e3


for sh in shapes:
    a = run(*sh, False)
    b = run(*sh, True)
    print(f"{sh[0]:20s} NCHW {a:9.2f} ms   channels_last {b:9.2f} ms", flush=True)
