"""turtle_train_gemm with per-image weights vs torch, over small-K / wide-N shapes (GPU box)."""
import sys
import torch
sys.path.insert(0, ".")
from turtlevsr_amd.train_ops import _gemm_rows, _rgemm_rows

torch.manual_seed(0)
for dt in (torch.float32, torch.bfloat16):
    for (nimg, m, K, N) in [(1, 16, 16, 16384), (1, 16, 16, 8192), (2, 16, 16, 8192), (4, 16, 16, 8192), (1, 16, 16, 4096),
                            (2, 32, 16, 16384), (1, 64, 16, 16384), (1, 16, 32, 16384), (1, 16, 128, 16)]:
        x = torch.randn(nimg * m, K, device="cuda").to(dt)
        w = torch.randn(nimg, N, K, device="cuda").to(dt)
        y = _gemm_rows(x, w).float()
        ref = torch.einsum("imk,ink->imn", x.float().view(nimg, m, K), w.float()).reshape(nimg * m, N)
        print(str(dt)[6:], (nimg, m, K, N), "gemm max err", float((y - ref).abs().max()), float(ref.abs().max()))
