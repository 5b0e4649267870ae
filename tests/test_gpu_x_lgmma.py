"""The line-graph attention on the matrix cores (csrc/lgmma.hip, bf16 storage, config C3) against the
VALU bf16 kernels (lgconv.hip) on the same operands: the products round q, u and alpha to bf16 (as the
reference's autocast holds them, train.py:632-636), so the comparison is within bf16 tolerances; the
dropout masks are the same hash, the softmax statistics fp32."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"

DEGREES = {
    "mp_mix": [132] * 40 + [11 * k for k in range(1, 12) for _ in range(4)],
    "ragged": [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 0, 13, 200, 17, 0, 31, 64, 65, 3, 1, 15, 16, 33],
    "empty_edges": [0, 0, 0],
}


def _nrel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp(min=1e-30))


def _case(degs, seed, with_wbar, D=256, H=4):
    from alignn_mi355x import ops
    g = torch.Generator().manual_seed(seed)
    degs = torch.as_tensor(degs)
    n = degs.numel()
    dst = torch.repeat_interleave(torch.arange(n), degs)
    src = torch.randint(0, n, (dst.numel(),), generator=g)
    csr = ops.GraphCSR(torch.stack([src, dst]).to(DEV), n)
    m = dst.numel()
    r = lambda *s: (torch.randn(*s, generator=g) * 0.5).to(DEV)  # noqa: E731
    QKV = r(n, 3 * D)
    t = dict(QKV=QKV, KV16=QKV[:, D:].contiguous().bfloat16(), U=r(n, H, D), F16=r(max(m, 1), D).bfloat16(),
             wbar=r(D) if with_wbar else None)
    return csr, m, t


def _fwd(fn, csr, t, drop, D=256, H=4):
    n = csr.n
    outs = dict(aggV=torch.empty(n, D, device=DEV), S=torch.empty(n, H, D, device=DEV),
                sumA=torch.empty(n, H, device=DEV), mstat=torch.empty(n, H, device=DEV),
                den=torch.empty(n, H, device=DEV))
    fn(csr, D, H, t["QKV"], t["KV16"], t["U"], t["wbar"], t["F16"], outs["aggV"], outs["S"], outs["sumA"],
       outs["mstat"], outs["den"], drop, 77)
    torch.cuda.synchronize()
    return outs


@pytest.mark.parametrize("drop", [0.0, 0.15])
@pytest.mark.parametrize("degs", list(DEGREES))
def test_mfma_forward_matches_valu_bf16_kernel(degs, drop):
    from alignn_mi355x import ops
    for seed, with_wbar in enumerate((True, False)):
        csr, m, t = _case(DEGREES[degs], 70 + seed, with_wbar)
        a = _fwd(ops.lg_fwd_mfma, csr, t, drop)
        b = _fwd(ops.lg_fwd_bf16, csr, t, drop)
        for k in ("aggV", "S", "sumA"):
            assert torch.isfinite(a[k]).all(), k
            assert _nrel(a[k], b[k]) < 2e-2, (k, _nrel(a[k], b[k]))
        fin = torch.isfinite(b["mstat"])
        assert torch.equal(fin, torch.isfinite(a["mstat"]))
        if fin.any():
            assert float((a["mstat"][fin] - b["mstat"][fin]).abs().max()) < 5e-2
        assert _nrel(a["den"], b["den"]) < 5e-2


def test_mfma_forward_is_deterministic():
    from alignn_mi355x import ops
    csr, m, t = _case(DEGREES["mp_mix"], 5, True)
    a = _fwd(ops.lg_fwd_mfma, csr, t, 0.15)
    b = _fwd(ops.lg_fwd_mfma, csr, t, 0.15)
    for k in a:
        assert torch.equal(a[k], b[k]), k


def _bwd(fn, csr, m, t, fo, drop, D=256, H=4):
    n = csr.n
    g = torch.Generator().manual_seed(99)
    Vd = (torch.randn(n, H, D, generator=g) * 0.5).to(DEV)
    dout = (torch.randn(n, D, generator=g) * 0.5).to(DEV)
    outs = dict(dq=torch.full((n, D), float("nan"), device=DEV), Sz=torch.empty(n, H, D, device=DEV),
                sigz=torch.empty(n, H, device=DEV), dz=torch.zeros(max(m, 1), H, device=DEV),
                al=torch.zeros(max(m, 1), H, device=DEV))
    fn(csr, D, H, t["QKV"], t["KV16"], t["U"], Vd, t["wbar"], t["F16"], dout, fo["aggV"], fo["mstat"], fo["den"],
       outs["dq"], outs["Sz"], outs["sigz"], outs["dz"], outs["al"], drop, 77)
    torch.cuda.synchronize()
    return outs


@pytest.mark.parametrize("drop", [0.0, 0.15])
@pytest.mark.parametrize("degs", list(DEGREES))
def test_mfma_backward_matches_valu_bf16_kernel(degs, drop):
    """Both backwards on the SAME forward statistics (the VALU forward's), so the comparison isolates
    the backward's own bf16 rounding (q, u, Vd, dout in the products, dz in the sums)."""
    from alignn_mi355x import ops
    for seed, with_wbar in enumerate((True, False)):
        csr, m, t = _case(DEGREES[degs], 80 + seed, with_wbar)
        fo = _fwd(ops.lg_fwd_bf16, csr, t, drop)
        a = _bwd(ops.lg_bwd_dst_mfma, csr, m, t, fo, drop)
        b = _bwd(ops.lg_bwd_dst_bf16, csr, m, t, fo, drop)
        for k in ("dq", "Sz", "sigz", "dz", "al"):
            assert torch.isfinite(a[k]).all(), k
            if m == 0 and k in ("dz", "al"):
                continue
            assert _nrel(a[k], b[k]) < 3e-2, (k, _nrel(a[k], b[k]))
