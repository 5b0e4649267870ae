"""The line convs' edge features recomputed inside the attention kernels (csrc/lgconv.hip XF path,
alignn_lg_fwd_x / alignn_lg_bwd_dst_x, and alignn_enc_bwd_bf16 without F16): the angle encoder's
hidden layer f = relu(x W1^T + b1) (train.py:358-364, :553-556) is recomputed from the 11 raw inputs
per edge group on the matrix cores instead of being materialised by linear_smallk and re-read.

* fp32: against the streamed-row kernels on the materialised layer (linear_smallk output): bitwise
  forward; the target-side backward runs one group in flight against the streamed kernel's two, and
  the compiler contracts the per-edge softmax terms differently (1-ulp differences, DESIGN §9 round
  4): 1e-6 of each output's largest magnitude.  (The bf16 form runs on the matrix cores with
  autocast's operand rounding: tests/test_gpu_x_lgmx.py.)
* The whole step: recompute_angle on vs off — loss and gradients (C2 fp32, B = 4: the same
  arithmetic; C3 bf16, B = 16: both layers are autocast's bf16(x) bf16(W1)^T + bf16(b1) with fp32
  accumulation, on different matrix-core shapes (16x16x32 in lgmx.hip, 32x32x16 in
  linear_smallk_bf16), so the two steps agree to bf16 rounding of the hidden layer).
"""
import pytest
import torch

from test_gpu_x_lg3 import DEGREES, _case
from test_gpu_x_pending import _rel

pytestmark = pytest.mark.gpu
DEV = "cuda"
D, H = 256, 4


def _ops():
    from alignn_mi355x import ops
    return ops


def _xcase(degs, seed, with_wbar):
    ops = _ops()
    csr, m, t = _case(H, degs, seed, with_wbar)
    csr._sched = None
    csr.policy = ops.SchedulePolicy(wave_items=True, xcd_items=True)
    g = torch.Generator().manual_seed(seed + 1000)
    xbuf = torch.empty(max(m, 1), 12, device=DEV)
    x = xbuf[:, :11]
    x.copy_(torch.randn(max(m, 1), 11, generator=g).to(DEV))
    W1 = (torch.randn(D, 11, generator=g) * 0.4).to(DEV)
    b1 = (torch.randn(D, generator=g) * 0.1).to(DEV)
    return csr, m, t, x, W1, b1


def _outs(n, m):
    o = dict(outp=torch.empty(n, D, device=DEV), S=torch.empty(n, H, D, device=DEV))
    for k in ("sumA", "mstat", "den", "sigz"):
        o[k] = torch.empty(n, H, device=DEV)
    o["dq"] = torch.full((n, D), float("nan"), device=DEV)
    o["Sz"] = torch.empty(n, H, D, device=DEV)
    o["dz"], o["al"] = torch.empty(max(m, 1), H, device=DEV), torch.empty(max(m, 1), H, device=DEV)
    return o


def _streamed(csr, m, t, x, W1, b1, drop, bf16):
    ops = _ops()
    n = csr.n
    o = _outs(n, m)
    QKV = t["QKVR"]
    if bf16:
        F16 = torch.empty(max(m, 1), D, device=DEV, dtype=torch.bfloat16)
        ops.linear_smallk_bf16(x, W1, b1, F16, relu=True)
        KV16 = ops.cast_bf16(QKV[:, :3 * D].contiguous())[:, D:3 * D]
        ops.lg_fwd_bf16(csr, D, H, QKV, KV16, t["U"], t["wbar"], F16, o["outp"], o["S"], o["sumA"], o["mstat"],
                        o["den"], drop, 77)
        ops.lg_bwd_dst_bf16(csr, D, H, QKV, KV16, t["U"], t["Vd"], t["wbar"], F16, t["dout"], o["outp"], o["mstat"],
                            o["den"], o["dq"], o["Sz"], o["sigz"], o["dz"], o["al"], drop, 77)
    else:
        F = torch.empty(max(m, 1), D, device=DEV)
        ops.linear_smallk(x, W1, b1, F, relu=True)
        assert csr.family(D, H, F) == 3
        ops.tconv_fwd(csr, D, H, QKV, t["U"], t["wbar"], F, None, o["outp"], o["S"], o["sumA"], o["mstat"], o["den"],
                      drop, 77)
        ops.tconv_bwd_dst(csr, D, H, QKV, t["U"], t["Vd"], t["wbar"], F, None, t["dout"], o["outp"], o["mstat"],
                          o["den"], o["dq"], o["Sz"], o["sigz"], o["dz"], o["al"], None, 0, drop, 77)
    torch.cuda.synchronize()
    return o


def _recomputed(csr, m, t, x, W1, b1, drop, bf16):
    ops = _ops()
    n = csr.n
    o = _outs(n, m)
    QKV = t["QKVR"]
    KV16 = ops.cast_bf16(QKV[:, :3 * D].contiguous())[:, D:3 * D] if bf16 else None
    ops.lg_fwd_x(csr, D, H, QKV, KV16, t["U"], t["wbar"], x, W1, b1, o["outp"], o["S"], o["sumA"], o["mstat"],
                 o["den"], drop, 77)
    ops.lg_bwd_dst_x(csr, D, H, QKV, KV16, t["U"], t["Vd"], t["wbar"], x, W1, b1, t["dout"], o["outp"], o["mstat"],
                     o["den"], o["dq"], o["Sz"], o["sigz"], o["dz"], o["al"], drop, 77)
    torch.cuda.synchronize()
    return o


FWD = ("outp", "S", "sumA", "mstat", "den")


@pytest.mark.parametrize("bf16", [False])
@pytest.mark.parametrize("drop", [0.0, 0.15])
@pytest.mark.parametrize("degs", list(DEGREES))
def test_recomputed_edge_features_match_streamed_rows(bf16, drop, degs):
    for seed, with_wbar in enumerate((True, False)):
        csr, m, t, x, W1, b1 = _xcase(DEGREES[degs], 60 + seed, with_wbar)
        a = _streamed(csr, m, t, x, W1, b1, drop, bf16)
        b = _recomputed(csr, m, t, x, W1, b1, drop, bf16)
        for k in a:
            if k in ("dz", "al"):
                if m == 0:
                    continue
                a[k], b[k] = a[k][:m], b[k][:m]
            if bf16 or k in FWD:
                assert torch.equal(a[k], b[k]), (k, bf16, drop, degs, seed, _rel(b[k], a[k]))
            else:
                assert _rel(b[k], a[k]) < 1e-6, (k, drop, degs, seed)


def test_recompute_rejects_unsupported_shapes():
    ops = _ops()
    csr, m, t, x, W1, b1 = _xcase(DEGREES["mp_mix"], 3, True)
    o = _outs(csr.n, m)
    bad_x = torch.empty(m, 11, device=DEV)   # rows of 11 floats (not the padded 12)
    with pytest.raises(ValueError):
        ops.lg_fwd_x(csr, D, H, t["QKVR"], None, t["U"], None, bad_x, W1, b1, o["outp"], o["S"], o["sumA"],
                     o["mstat"], o["den"], 0.0, 1)
    with pytest.raises(ValueError):
        ops.lg_fwd_x(csr, D, H, t["QKVR"], None, t["U"], None, x, W1[:, :10].contiguous(), b1, o["outp"], o["S"],
                     o["sumA"], o["mstat"], o["den"], 0.0, 1)


@pytest.mark.parametrize("precision,B", [("fp32", 4), ("bf16", 16)])
def test_step_with_recomputed_angle_layer(precision, B):
    """The training step's loss and gradients with recompute_angle on (the default) and off.  fp32: the
    forward is bitwise (same attention arithmetic on bitwise the same edge features), gradients to
    fp32 summation order of the target-side backward (one group in flight vs two).  bf16: the two
    hidden layers differ by bf16 rounding (fp32 sums of the same bf16 products in another order), and
    the attention arithmetic differs (matrix-core products with bf16 Q / U operands vs fp32 VALU):
    loss to 1e-2, every gradient within 5e-2 normwise and cosine > 0.998 (gradients that are zero up to
    rounding: both below 1e-4 of the largest)."""
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    res = {}
    batch = mp_like_batch(B).to(DEV)
    for on in (True, False):
        torch.manual_seed(0)
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(DEV)
        tr = A.FusedTrainer(model, precision=precision)
        model._engine.recompute_angle = on
        model._engine.recompute_angle_bf16 = on
        assert model._engine._angle_xf(A.engine.batch_cache(batch), 256) == on
        loss = tr.forward_backward(batch, 5).clone()
        torch.cuda.synchronize()
        res[on] = (loss, {k: v.clone() for k, v in tr.st.G.named.items()})
    (l1, g1), (l0, g0) = res[True], res[False]
    if precision == "bf16":
        assert abs(float(l1) - float(l0)) <= 1e-2 * abs(float(l0)), (float(l1), float(l0))
        top = max(float(v.double().norm()) for v in g0.values())
        for k in g0:
            a, b = g1[k].double().flatten(), g0[k].double().flatten()
            nb = float(b.norm())
            if nb <= 1e-4 * top:
                # analytically zero up to rounding (the key bias: a per-target constant shift of every
                # score, which the softmax cancels) — its rounding noise has no direction to compare
                assert float(a.norm()) <= 1e-4 * top, k
                continue
            assert float((a - b).norm()) <= 5e-2 * nb, (k, float((a - b).norm()) / nb)
            assert float(a @ b) >= 0.998 * float(a.norm()) * nb, k
        return
    assert torch.equal(l1, l0)
    gmax = max(float(v.abs().max()) for v in g0.values())
    for k in g0:
        assert float((g1[k] - g0[k]).abs().max()) <= 1e-5 * gmax, k
