"""Probe: vendor GEMM (torch.matmul -> hipBLASLt/rocBLAS) time for the Turtle 1080p GEMM shapes,
bf16, D = A W^T (+ C), as a yardstick for the in-tree kernels (tools/kbench)."""
import torch

shapes = [(130560, 1280, 256, 0, "L3 project_in"), (130560, 768, 256, 0, "L3 qkv"),
          (130560, 256, 640, 1, "L3 project_out +res"), (130560, 256, 256, 1, "L3 W_eff +res"),
          (32640, 2560, 512, 0, "latent project_in"), (32640, 1536, 512, 0, "latent qkv"),
          (32640, 512, 1280, 1, "latent project_out +res"), (32640, 512, 512, 1, "latent W_eff +res"),
          (522240, 256, 128, 0, "L2 conv4"), (522240, 128, 256, 1, "L2 conv5 +res"),
          (2088960, 64, 128, 1, "L1 conv5 +res")]
dev = "cuda"
for M, N, K, res, tag in shapes:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
    c = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
    f = (lambda: torch.addmm(c, a, w.t())) if res else (lambda: a @ w.t())
    for _ in range(3):
        f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        f()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / 20
    byt = 2 * (M * K + M * N * (2 if res else 1))
    print(f"{tag:26s} M={M:8d} N={N:5d} K={K:5d}: {us:8.1f} us  {2*M*N*K/us/1e6:7.1f} TF/s  {byt/us/1e3:7.0f} GB/s", flush=True)
