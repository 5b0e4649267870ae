"""The bf16 line-graph attention on the matrix cores (csrc/lgmx.hip; alignn_lg_fwd_x / alignn_lg_bwd_dst_x
with bf16 K|V, config C3) and the deferred encoder backward that recomputes its ReLU mask the same way
(alignn_enc_bwd_bf16 without F16).

* Against a float64 restatement of PyG's TransformerConv attention (oracle/pyg_ref.py's
  formula with the edge-feature algebra of DESIGN §3) on the operands as the matrix cores take them:
  the angle encoder's hidden layer as autocast computes it (train.py:554 under :636: x, W1 and b1
  rounded to bf16, fp32 accumulation, the output rounded to bf16), Q / U / Vd / dout rounded to bf16
  where they enter a product, K and V the bf16 copies.  What remains is fp32 accumulation order and the
  attention weights' hi + lo bf16 split (~2^-17): 2e-4 of each output's largest magnitude.
* With dropout, against the streamed-row bf16 kernels (lgconv.hip) fed the same hidden layer: the same
  masks (one counter hash per (edge, head)) — a misplaced mask moves outputs by O(1); the remaining
  difference is those kernels' fp32 Q / U operands (bf16 rounding): 2e-2.
* The encoder backward's recomputed mask against the mask read from the stored layer.
"""
import pytest
import torch

from test_gpu_x_lg3 import DEGREES
from test_gpu_x_pending import _rel
from test_gpu_x_recompute import _outs, _xcase

pytestmark = pytest.mark.gpu
DEV = "cuda"
D, H, C = 256, 4, 64


def _ops():
    from alignn_mi355x import ops
    return ops


def _bf(t):
    return t.to(torch.bfloat16).double()


def autocast_hidden(x, W1, b1):
    """bf16(relu(bf16(x) bf16(W1)^T + bf16(b1))) — the angle encoder's first Linear + ReLU under autocast."""
    pre = _bf(x) @ _bf(W1).t() + _bf(b1)
    return torch.relu(pre).to(torch.bfloat16)


def _mx(csr, m, t, x, W1, b1, drop):
    ops = _ops()
    o = _outs(csr.n, m)
    QKV = t["QKVR"]
    KV16 = ops.cast_bf16(QKV[:, :3 * D].contiguous())[:, D:3 * D]
    ops.lg_fwd_x(csr, D, H, QKV, KV16, t["U"], t["wbar"], x, W1, b1, o["outp"], o["S"], o["sumA"], o["mstat"],
                 o["den"], drop, 77)
    ops.lg_bwd_dst_x(csr, D, H, QKV, KV16, t["U"], t["Vd"], t["wbar"], x, W1, b1, t["dout"], o["outp"], o["mstat"],
                     o["den"], o["dq"], o["Sz"], o["sigz"], o["dz"], o["al"], drop, 77)
    torch.cuda.synchronize()
    return o, KV16


def _reference(t, x, W1, b1, KV16, outp, n, m):
    """Float64 forward + target-side backward (dropout 0) on the matrix-core operands."""
    src, dst = t["src"].to(DEV), t["dst"].to(DEV)
    F = autocast_hidden(x[:m], W1, b1).double()
    Q = _bf(t["QKVR"][:, :D]).view(n, H, C)
    K = KV16[:, :D].double().view(n, H, C)
    V = KV16[:, D:].double().view(n, H, C)
    U, Vd = _bf(t["U"]), _bf(t["Vd"])
    dout = t["dout"].double().view(n, H, C)
    wb = t["wbar"].double().view(H, C) if t["wbar"] is not None else torch.zeros(H, C, dtype=torch.float64, device=DEV)
    q32 = t["QKVR"][:, :D].double().view(n, H, C)
    raw = (Q[dst] * K[src]).sum(-1) + (U[dst] * F[:, None, :]).sum(-1) + (q32[dst] * wb).sum(-1)
    z = raw / C ** 0.5
    zmax = torch.full((n, H), float("-inf"), dtype=torch.float64, device=DEV).scatter_reduce(
        0, dst[:, None].expand(-1, H), z, "amax")
    ex = torch.exp(z - zmax[dst])
    den = torch.zeros(n, H, dtype=torch.float64, device=DEV).index_add(0, dst, ex) + 1e-16
    alpha = ex / den[dst]
    aggV = torch.zeros(n, H, C, dtype=torch.float64, device=DEV).index_add(0, dst, alpha[:, :, None] * V[src])
    S = torch.zeros(n, H, D, dtype=torch.float64, device=DEV).index_add(0, dst, alpha[:, :, None] * F[:, None, :])
    sumA = torch.zeros(n, H, dtype=torch.float64, device=DEV).index_add(0, dst, alpha)
    # backward: dalpha = <dout_h, V_s,h> + <Vd_h, f> + <w̄_h, dout_h>; dz = alpha (dalpha - <dout, out>) / sqrt(C)
    O = _bf(t["dout"]).view(n, H, C)
    dal = (O[dst] * V[src]).sum(-1) + (Vd[dst] * F[:, None, :]).sum(-1) + (dout[dst] * wb).sum(-1)
    pdl = (dout * outp.double().view(n, H, C)).sum(-1)
    dz = alpha * (dal - pdl[dst]) / C ** 0.5
    dq = torch.zeros(n, H, C, dtype=torch.float64, device=DEV).index_add(0, dst, dz[:, :, None] * K[src])
    Sz = torch.zeros(n, H, D, dtype=torch.float64, device=DEV).index_add(0, dst, dz[:, :, None] * F[:, None, :])
    sigz = torch.zeros(n, H, dtype=torch.float64, device=DEV).index_add(0, dst, dz)
    return dict(outp=aggV.reshape(n, D), S=S, sumA=sumA, mstat=zmax, den=den, dz=dz, al=alpha,
                dq=dq.reshape(n, D), Sz=Sz, sigz=sigz)


@pytest.mark.parametrize("degs", list(DEGREES))
def test_mx_kernels_vs_float64_reference(degs):
    for seed, with_wbar in enumerate((True, False)):
        csr, m, t, x, W1, b1 = _xcase(DEGREES[degs], 90 + seed, with_wbar)
        o, KV16 = _mx(csr, m, t, x, W1, b1, 0.0)
        ref = _reference(t, x, W1, b1, KV16, o["outp"], csr.n, m)
        for k, r in ref.items():
            got = o[k]
            if k in ("dz", "al"):
                if m == 0:
                    continue
                got = got[:m]
            # the backward's <dout, out> uses the kernel's forward output, so dz and its sums see
            # the forward's error once more
            tol = 2e-4 if k in ("outp", "S", "sumA", "mstat", "den", "al") else 5e-4
            assert _rel(got, r) < tol, (k, degs, seed, _rel(got, r))


@pytest.mark.parametrize("degs", ["mp_mix", "ragged"])
def test_mx_kernels_dropout_masks_match_streamed_rows(degs):
    ops = _ops()
    csr, m, t, x, W1, b1 = _xcase(DEGREES[degs], 7, True)
    o, KV16 = _mx(csr, m, t, x, W1, b1, 0.15)
    F16 = torch.empty(max(m, 1), D, device=DEV, dtype=torch.bfloat16)
    F16[:m] = autocast_hidden(x[:m], W1, b1)
    a = _outs(csr.n, m)
    QKV = t["QKVR"]
    ops.lg_fwd_bf16(csr, D, H, QKV, KV16, t["U"], t["wbar"], F16, a["outp"], a["S"], a["sumA"], a["mstat"], a["den"],
                    0.15, 77)
    ops.lg_bwd_dst_bf16(csr, D, H, QKV, KV16, t["U"], t["Vd"], t["wbar"], F16, t["dout"], a["outp"], a["mstat"],
                        a["den"], a["dq"], a["Sz"], a["sigz"], a["dz"], a["al"], 0.15, 77)
    torch.cuda.synchronize()
    for k in a:
        x_, y_ = o[k], a[k]
        if k in ("dz", "al"):
            x_, y_ = x_[:m], y_[:m]
            # a mask in the wrong place zeroes a different weight: the zero patterns must agree
            assert torch.equal(x_ == 0, y_ == 0), k
        assert _rel(x_, y_) < 2e-2, (k, _rel(x_, y_))


@pytest.mark.parametrize("n,L,src", [(40, 4, "torch"), (9, 2, "torch"), (40, 4, "mx"), (300, 4, "mx")])
def test_enc_bwd_bf16_mask_recomputed_matches_stored_layer(n, L, src):
    """alignn_enc_bwd_bf16 with its mask recomputed on the matrix cores (F16 NULL) against the mask read
    from the stored hidden layer: the same products, the same mask.  'mx': the layer from
    ops.linear_smallk_bf16 (config C3's stored layer), whose pre-activation is the recompute's bit for
    bit — the engine then takes the recompute (engine._backward_tail).  'torch': torch's autocast
    arithmetic (a pre-activation within one rounding of 0 could sit on the other side; the random case
    has none)."""
    from test_gpu_x_encbwd import _case as eb_case
    ops = _ops()
    csr, x, W1, b1, U, Vd, dz, al = eb_case(n, 256, 4, L, 11, seed=n + L)
    if src == "mx":
        F16 = torch.empty(x.size(0), 256, device=DEV, dtype=torch.bfloat16)
        ops.linear_smallk_bf16(x, W1, b1, F16, relu=True)
    else:
        F16 = autocast_hidden(x, W1, b1).contiguous()
    dW1a, db1a = torch.empty(256, 11, device=DEV), torch.empty(256, device=DEV)
    dW1b, db1b = torch.empty(256, 11, device=DEV), torch.empty(256, device=DEV)
    ops.enc_bwd(csr, x, W1, b1, U, Vd, dz, al, dW1a, db1a, F=F16)
    ops.enc_bwd(csr, x, W1, b1, U, Vd, dz, al, dW1b, db1b, bf16=True)
    torch.cuda.synchronize()
    assert torch.equal(dW1a, dW1b) and torch.equal(db1a, db1b)
