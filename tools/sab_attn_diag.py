"""SAB attention core on HIP vs the ATen formulation at the training graph's shapes (GPU box)."""
import sys
import torch
sys.path.insert(0, ".")
from turtlevsr_amd.train_ops import HipOps
from turtlevsr_amd.train import TrainGraph

torch.manual_seed(0)
dev = "cuda"
for (b, n, tw, g, c, ws, t) in [(1, 16, 4, 128, 64, 16, 1), (1, 16, 4, 128, 64, 16, 2), (2, 16, 4, 256, 128, 8, 2), (2, 64, 8, 32, 4, 4, 3)]:
    D = ws * ws * c
    q = torch.nn.functional.normalize(torch.randn(b, n, g, device=dev), dim=-1)
    K = torch.nn.functional.normalize(torch.randn(b, t, n, g, device=dev), dim=-1)
    v = torch.randn(b, c, int(n ** 0.5) * ws, int(n ** 0.5) * ws, device=dev)
    VT = TrainGraph._dilated_t(v, ws).expand(b, t, D, n).contiguous()
    vt = TrainGraph._dilated(v, ws).reshape(b, 1, n, D).expand(b, t, n, D)
    print("dilated_t == dilated^T:", torch.equal(VT.transpose(-1, -2), vt))
    temp = torch.full((1, 1, 1), 0.9, device=dev)
    o = HipOps.sab_attention(q, K, VT, temp, tw, 4)
    s2 = (q[:, None] @ K.transpose(-1, -2)) * temp
    qi = torch.arange(n, device=dev)
    ball = (((qi[:, None] // tw - qi[None, :] // tw).abs() + (qi[:, None] % tw - qi[None, :] % tw).abs()) <= 4).float()
    top = torch.zeros_like(s2).scatter_(-1, torch.topk(s2, 5, dim=-1).indices, 1.0)
    se = s2 * (top + ball)
    zero = se == 0
    p = torch.softmax(se.masked_fill(zero, float("-inf")), dim=-1).masked_fill(zero, 0.0)
    o2 = (p / p.sum(dim=-1, keepdim=True)) @ vt
    S = (q[:, None] @ K.transpose(-1, -2))
    print((b, n, tw, g, c, ws, t), "max|o - o2|", float((o - o2).abs().max()), "max|o2|", float(o2.abs().max()))
