"""Diagnostics: per-parameter gradient error of the engine vs the fp64 oracle (and the fp32
oracle's own error), for one full-size batch.  python tools/diag_parity.py [num_graphs] [lg_offset]"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "gnn-elasticity-predictor_amd"), REPO]
import alignn_mi355x as A  # noqa: E402
from alignn_mi355x.synthetic import mp_like_batch  # noqa: E402
from oracle import model_ref  # noqa: E402
from oracle.pyg_ref import RefData  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
mode = sys.argv[2] if len(sys.argv) > 2 else "num_nodes"
torch.manual_seed(5)
model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.0), 2)
st = {k: v.detach().clone() for k, v in model.state_dict().items()}
cpu_batch = mp_like_batch(B, lg_offset=mode)


def oracle(dt):
    b = RefData(**{k: getattr(cpu_batch, k) for k in cpu_batch.keys()})
    for k in ("x", "edge_attr", "lg_edge_attr", "global_x", "sg_one_hot", "y"):
        setattr(b, k, getattr(b, k).to(dt))
    b.num_graphs = B
    ps = {k: v.to(dt).clone().requires_grad_(True) for k, v in st.items()}
    ret = {}
    mean, logvar = model_ref.hetero_forward(ps, b, 4, retain=ret)
    RET[dt] = ret
    tz = model_ref.log_transform(b.y.view(B, -1), (4.3228, 3.5567), (0.9051, 0.9405))
    model_ref.hetero_loss(mean, logvar, tz, 0.1).backward()
    return mean.detach(), {k: v.grad for k, v in ps.items() if v.grad is not None}


RET = {}
m64, g64 = oracle(torch.float64)
m32, g32 = oracle(torch.float32)
model.to("cuda").train()
model._engine.debug = {}
_orig_fwd = model._engine.forward


def _fwd(*a, **k):
    out, ctx = _orig_fwd(*a, **k)
    CTX.append(ctx)
    return out, ctx


CTX = []
model._engine.forward = _fwd
b = cpu_batch.to("cuda")
mean, logvar = model(b)
y = b.y.view(B, -1)
tz = (torch.log(y) - torch.tensor([4.3228, 3.5567], device="cuda")) / torch.tensor([0.9051, 0.9405], device="cuda")
lv = torch.clamp(logvar, min=-2.9)
((0.5 * (lv + (mean - tz) ** 2 / torch.exp(lv))).mean(1).mean() + 0.1 * (0.5 * lv).pow(2).mean()).backward()
gmax = max(float(v.abs().max()) for v in g64.values())


def rel(a, b):
    return float((a.double().cpu() - b).abs().max() / max(float(b.abs().max()), 1e-3 * gmax))


print("mean rel err: engine", rel(mean.detach(), m64), "oracle32", rel(m32, m64))
rows = []
for k, p in model.named_parameters():
    if k in g64:
        rows.append((rel(p.grad, g64[k]), rel(g32[k], g64[k]), k))
for e, e32, k in sorted(rows, reverse=True)[:25]:
    print(f"{e:9.2e} {e32:9.2e} {k}")
dbg = model._engine.debug
for l in range(4, 0, -1):
    for name, key in ((f"dh{l}", f"h{l}"), (f"de{l}", f"e{l}")):
        ref = RET[torch.float64][key].grad
        r32 = RET[torch.float32][key].grad
        got = dbg[name]
        err = (got.double().cpu() - ref).abs()
        print(f"{name}: engine {float(err.max() / ref.abs().max()):.2e} oracle32 "
              f"{float((r32.double() - ref).abs().max() / ref.abs().max()):.2e}  worst row {int(err.max(1).values.argmax())}")

ref = RET[torch.float64]["e0"].grad
got = dbg["de0"].double().cpu()
err = (got - ref).abs().max(1).values / ref.abs().max()
deg = torch.bincount(cpu_batch.lg_edge_index[1].cpu(), minlength=cpu_batch.edge_index.size(1))
print("de0 engine", float(err.max()), "rows with lg in-edges", float(err[deg > 0].max()), "without", float(err[deg == 0].max()))
srcdeg = torch.bincount(cpu_batch.lg_edge_index[0].cpu(), minlength=cpu_batch.edge_index.size(1))
print("rows as lg source", float(err[srcdeg > 0].max()), "never source", float(err[srcdeg == 0].max()))
worst = int(err.argmax()); print("worst row", worst, "deg", int(deg[worst]), "srcdeg", int(srcdeg[worst]))
c = CTX[0].edge[0]
D = 256
R = c.R
y = c.beta[:, None] * R + (1 - c.beta[:, None]) * c.outp
mu = y.mean(1)
var = ((y - mu[:, None]) ** 2).mean(1)
print("edge0 mu err", float((mu - c.mu).abs().max()), "rstd rel err", float(((1 / torch.sqrt(var + 1e-5)) / c.rstd - 1).abs().max()))
print("edge0 outp isolated rows max", float(c.outp[(deg == 0).cuda()].abs().max()))
lg = torch.sigmoid((torch.cat([c.outp, R, c.outp - R], 1) * model.base.edge_blocks[0].conv.lin_beta.weight).sum(1))
print("edge0 beta err", float((lg - c.beta).abs().max()))
print("rstd range", float(c.rstd.min()), float(c.rstd.max()), "worst row rstd", float(c.rstd[worst]), "var", float(var[worst]))
# replicate gate/LN backward of edge block 0 in fp64 from saved state
blk = model.base.edge_blocks[0]
dXn = dbg["de1"].double()
o, Rr, b_ = c.outp.double(), R.double(), c.beta.double()[:, None]
yy = b_ * Rr + (1 - b_) * o
yh = (yy - c.mu.double()[:, None]) * c.rstd.double()[:, None]
ln = yh * blk.norm.weight.double() + blk.norm.bias.double()
gl = dXn * (ln > 0)
gyh = gl * blk.norm.weight.double()
dy = c.rstd.double()[:, None] * (gyh - gyh.mean(1, keepdim=True) - yh * (gyh * yh).mean(1, keepdim=True))
wb = blk.conv.lin_beta.weight.double().view(-1)
dl = (dy * (Rr - o)).sum(1, keepdim=True) * b_ * (1 - b_)
dR = b_ * dy + dl * (wb[D:2 * D] - wb[2 * D:])
de0_iso = dXn + dR @ blk.conv.lin_skip.weight.double()
iso = (deg == 0).cuda() & (srcdeg == 0).cuda()
ref = RET[torch.float64]["e0"].grad.cuda()
print("replicated iso de0 vs oracle", float((de0_iso[iso] - ref[iso]).abs().max() / ref.abs().max()))
print("engine iso de0 vs replicated", float((dbg["de0"].double()[iso] - de0_iso[iso]).abs().max() / ref.abs().max()))
print("worst row engine", dbg["de0"][worst, :4].tolist(), "oracle", ref[worst, :4].tolist(), "repl", de0_iso[worst, :4].tolist())
dXn = RET[torch.float64]["e1"].grad.cuda()
gl = dXn * (ln > 0)
gyh = gl * blk.norm.weight.double()
dy = c.rstd.double()[:, None] * (gyh - gyh.mean(1, keepdim=True) - yh * (gyh * yh).mean(1, keepdim=True))
dl = (dy * (Rr - o)).sum(1, keepdim=True) * b_ * (1 - b_)
dR = b_ * dy + dl * (wb[D:2 * D] - wb[2 * D:])
de0_iso2 = dXn + dR @ blk.conv.lin_skip.weight.double()
print("replicated(oracle de1) iso vs oracle de0", float((de0_iso2[iso] - ref[iso]).abs().max() / ref.abs().max()))
e1r = RET[torch.float64]["e1"].grad.cuda()
print("de1 iso rows: engine vs oracle rel-to-row", float(((dbg["de1"].double() - e1r).abs().max(1).values / e1r.abs().max(1).values.clamp(min=1e-30))[iso].max()))
