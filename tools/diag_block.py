"""Block-level gradient error of EdgeUpdateBlock / NodeUpdateBlock (engine vs fp64 oracle, plus the
fp32 oracle's own error) on a skewed graph.  python tools/diag_block.py [heavy_threshold]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "gnn-elasticity-predictor_amd"), REPO]
import alignn_mi355x as A  # noqa: E402
from alignn_mi355x import ops  # noqa: E402
from oracle.model_ref import edge_block, node_block  # noqa: E402

if len(sys.argv) > 1:
    ops.DEFAULT_SCHEDULE = ops.SchedulePolicy(heavy_threshold=int(sys.argv[1]))
torch.manual_seed(0)
D, H = 256, 4
n, m = 1000, 30000
g = torch.Generator().manual_seed(1)
ei = torch.stack([torch.randint(0, n, (m,), generator=g), torch.randint(0, 200, (m,), generator=g)])
blk = A.EdgeUpdateBlock(D, H, 0.0)
x = torch.randn(n, D, generator=g)
f = torch.randn(m, D, generator=g).relu()
w = torch.randn(n, D, generator=g)


def oracle(dt):
    xs, fs = x.to(dt).clone().requires_grad_(True), f.to(dt).clone().requires_grad_(True)
    ps = {f"e.{k}": v.detach().to(dt).clone().requires_grad_(True) for k, v in blk.state_dict().items()}
    out = edge_block(ps, "e.", xs, ei, fs, H)
    (out * w.to(dt)).sum().backward()
    return out.detach(), xs.grad, fs.grad, {k[2:]: v.grad for k, v in ps.items()}


o64, x64, f64, p64 = oracle(torch.float64)
o32, x32, f32, p32 = oracle(torch.float32)
blk.to("cuda")
xd, fd = x.cuda().requires_grad_(True), f.cuda().requires_grad_(True)
out = blk(xd, ei.cuda(), fd)
(out * w.cuda()).sum().backward()


def rel(a, b):
    return float((a.detach().double().cpu() - b).abs().max() / b.abs().max())


print("out", rel(out, o64), rel(o32, o64))
print("dx", rel(xd.grad, x64), rel(x32, x64))
print("df", rel(fd.grad, f64), rel(f32, f64))
for k, p in blk.named_parameters():
    print(f"{rel(p.grad, p64[k]):9.2e} {rel(p32[k], p64[k]):9.2e} {k}")
