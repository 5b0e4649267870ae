"""Deferred angle-encoder backward (encbwd.hip, alignn_enc_bwd_f32; the autograd backward of the
angle encoder's first Linear + ReLU, train.py:358-364, as reached from every EdgeUpdateBlock):
kernel vs an fp64 restatement on random line graphs (ragged and empty segments, target changes
inside a chunk, H*L = 1..16, kin 1..16), accumulate mode and determinism; then the engine with
``defer_angle_bwd`` on vs off: same loss bitwise, W1/b1 gradients equal up to summation order.  The
other gradients agree to fp32 rounding, not bitwise: without deferral the line-graph ``bwd_dst``
writes the [T, D] edge-feature gradient, which the single-wave-item kernels (lgconv.hip) do not, so
that configuration takes the tconv.hip kernel family, whose dQ/Sz sums run in another order."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


def _case(n, D, H, L, kin, seed):
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(seed)
    deg = torch.randint(0, 300, (n,), generator=g)
    deg[::5] = 0
    deg[1] = 1000  # one segment spanning several chunks
    dst = torch.repeat_interleave(torch.arange(n), deg)
    src = torch.randint(0, n, (dst.numel(),), generator=g)
    csr = ops.GraphCSR(torch.stack([src, dst]).to(DEV), n)
    T = dst.numel()
    ldx = (kin + 3) // 4 * 4
    xb = torch.randn(T, max(ldx, 4), generator=g).to(DEV)
    x = xb[:, :kin]
    W1 = torch.randn(D, kin, generator=g).to(DEV) * 0.5
    b1 = torch.randn(D, generator=g).to(DEV) * 0.5
    U = [torch.randn(n, H, D, generator=g).to(DEV) for _ in range(L)]
    Vd = [torch.randn(n, H, D, generator=g).to(DEV) for _ in range(L)]
    dz = [torch.randn(max(T, 1), H, generator=g).to(DEV) for _ in range(L)]
    al = [torch.randn(max(T, 1), H, generator=g).to(DEV) for _ in range(L)]
    return csr, x, W1, b1, U, Vd, dz, al


def _reference(csr, x, W1, b1, U, Vd, dz, al):
    """fp64 restatement; the ReLU mask from the forward's own fp32 kernel (linear_smallk)."""
    from alignn_mi355x import ops
    T = x.size(0)
    D = W1.size(0)
    h1 = torch.empty(T, D, device=DEV)
    ops.linear_smallk(x, W1, b1, h1, relu=True)
    d = csr.dst_at[:T].long()
    gsum = torch.zeros(T, D, dtype=torch.float64, device=DEV)
    for Ul, Vl, zl, al_l in zip(U, Vd, dz, al):
        gsum += torch.einsum("th,thd->td", zl[:T].double(), Ul[d].double())
        gsum += torch.einsum("th,thd->td", al_l[:T].double(), Vl[d].double())
    dpre = gsum * (h1 > 0).double()
    return dpre.t() @ x.double(), dpre.sum(0)


@pytest.mark.parametrize("n,D,H,L,kin", [(40, 256, 4, 4, 11), (33, 64, 4, 2, 7), (17, 32, 1, 1, 7),
                                         (25, 256, 8, 2, 16), (30, 128, 2, 8, 1), (9, 256, 4, 4, 12)])
def test_enc_bwd_matches_fp64(n, D, H, L, kin):
    from alignn_mi355x import ops
    csr, x, W1, b1, U, Vd, dz, al = _case(n, D, H, L, kin, seed=n * 31 + D + H + L + kin)
    dW1 = torch.full((D, kin), float("nan"), device=DEV)
    db1 = torch.full((D,), float("nan"), device=DEV)
    ops.enc_bwd(csr, x, W1, b1, U, Vd, dz, al, dW1, db1)
    rW, rb = _reference(csr, x, W1, b1, U, Vd, dz, al)
    assert _rel(dW1, rW) < 1e-5 and _rel(db1, rb) < 1e-5
    # accumulate adds exactly the same partial sums; repeated launches are bitwise equal
    dW2, db2 = dW1.clone(), db1.clone()
    ops.enc_bwd(csr, x, W1, b1, U, Vd, dz, al, dW2, db2, accumulate=True)
    assert torch.equal(dW2, dW1 + dW1) and torch.equal(db2, db1 + db1)
    dW3, db3 = torch.empty_like(dW1), torch.empty_like(db1)
    ops.enc_bwd(csr, x, W1, b1, U, Vd, dz, al, dW3, db3)
    assert torch.equal(dW3, dW1) and torch.equal(db3, db1)


@pytest.mark.parametrize("n,H,L,kin", [(40, 4, 4, 11), (25, 8, 2, 16), (30, 2, 8, 1), (17, 2, 3, 7), (9, 4, 2, 11)])
def test_enc_bwd_bf16_matches_fp64(n, H, L, kin):
    """bf16 storage (config C3): the matrix-core kernel (alignn_enc_bwd_bf16) against an fp64
    restatement of its arithmetic — [dz | alpha'], U/Vd, dpre and x rounded to bf16, the ReLU mask
    from the bf16 hidden layer — and against the fp32 kernel at bf16 tolerance."""
    from alignn_mi355x import ops
    D = 256
    csr, x, W1, b1, U, Vd, dz, al = _case(n, D, H, L, kin, seed=n * 17 + H + L + kin)
    T = x.size(0)
    f16 = torch.empty(T, D, dtype=torch.bfloat16, device=DEV)
    if kin <= ops.SMALLK_BF16_MAX:
        ops.linear_smallk_bf16(x, W1, b1, f16, relu=True)
    else:   # past the matrix-core Linear's one k step: torch's autocast arithmetic
        f16.copy_(torch.relu(x.bfloat16().double() @ W1.bfloat16().double().t() + b1.bfloat16().double())
                  .float().bfloat16())
    dW1 = torch.full((D, kin), float("nan"), device=DEV)
    db1 = torch.full((D,), float("nan"), device=DEV)
    ops.enc_bwd(csr, x, W1, b1, U, Vd, dz, al, dW1, db1, F=f16)
    bf = lambda t: t.to(torch.bfloat16).double()  # noqa: E731
    d = csr.dst_at[:T].long()
    g = torch.zeros(T, D, dtype=torch.float64, device=DEV)
    for Ul, Vl, zl, al_l in zip(U, Vd, dz, al):
        g += torch.einsum("th,thd->td", bf(zl[:T]), bf(Ul)[d]) + torch.einsum("th,thd->td", bf(al_l[:T]), bf(Vl)[d])
    dpre = bf(g.float() * (f16.float() > 0))
    rW, rb = dpre.t() @ bf(x), dpre.sum(0)
    nrel = lambda a, b: float((a.double() - b).norm() / b.norm())  # noqa: E731
    assert nrel(dW1, rW) < 2e-3 and nrel(db1, rb) < 2e-3
    # the fp32 VALU kernel (exact fp32 products, mask from the fp32 pre-activation) at bf16 tolerance:
    # autocast's bf16 x and W move pre-activations near 0 across the ReLU, so the masks differ too
    fW, fb = torch.empty_like(dW1), torch.empty_like(db1)
    ops.enc_bwd(csr, x, W1, b1, U, Vd, dz, al, fW, fb)
    assert nrel(dW1, fW.double()) < 5e-2 and nrel(db1, fb.double()) < 5e-2
    # accumulate adds exactly the same partial sums; repeated launches are bitwise equal
    dW2, db2 = dW1.clone(), db1.clone()
    ops.enc_bwd(csr, x, W1, b1, U, Vd, dz, al, dW2, db2, accumulate=True, F=f16)
    assert torch.equal(dW2, dW1 + dW1) and torch.equal(db2, db1 + db1)
    dW3, db3 = torch.empty_like(dW1), torch.empty_like(db1)
    ops.enc_bwd(csr, x, W1, b1, U, Vd, dz, al, dW3, db3, F=f16)
    assert torch.equal(dW3, dW1) and torch.equal(db3, db1)


def test_enc_bwd_empty_graph_and_rejects_unsupported():
    from alignn_mi355x import ops
    csr = ops.GraphCSR(torch.zeros(2, 0, dtype=torch.int64, device=DEV), 5)
    x = torch.zeros(0, 11, device=DEV)
    W1, b1 = torch.randn(64, 11, device=DEV), torch.randn(64, device=DEV)
    U = [torch.randn(5, 4, 64, device=DEV)]
    z = [torch.zeros(1, 4, device=DEV)]
    dW1, db1 = torch.full((64, 11), 3.0, device=DEV), torch.full((64,), 3.0, device=DEV)
    ops.enc_bwd(csr, x, W1, b1, U, U, z, z, dW1, db1)
    assert torch.equal(dW1, torch.zeros_like(dW1)) and torch.equal(db1, torch.zeros_like(db1))
    assert not ops.enc_bwd_ok(512, 4, 4, 11) and not ops.enc_bwd_ok(256, 4, 5, 11)
    assert not ops.enc_bwd_ok(256, 4, 4, 17)


@pytest.mark.parametrize("lg_offset", ["num_nodes", "num_edges"])
def test_engine_deferred_angle_backward(lg_offset):
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    res = []
    for defer in (False, True):
        torch.manual_seed(0)
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(DEV)
        model._engine.defer_angle_bwd = defer
        tr = A.FusedTrainer(model)
        b = mp_like_batch(4, lg_offset=lg_offset).to(DEV)
        loss = tr.forward_backward(b, 3).clone()
        torch.cuda.synchronize()
        res.append((loss, tr.st.grad.clone(), tr.st))
    (l0, g0, st), (l1, g1, _) = res
    assert torch.equal(l0, l1)
    P = st.P
    w1 = P.enc("angle", 0, "weight")
    b1 = P.enc("angle", 0, "bias")
    o_w, o_b = w1.storage_offset() - st.flat.storage_offset(), b1.storage_offset() - st.flat.storage_offset()
    sl = [slice(o_w, o_w + w1.numel()), slice(o_b, o_b + b1.numel())]
    for s_ in sl:
        assert _rel(g1[s_], g0[s_]) < 1e-5
    # per-parameter normwise agreement (different attention kernel families, see the module doc);
    # the key-bias gradients are exactly 0 in exact arithmetic (softmax is shift-invariant): both
    # sides must be rounding noise (< 1e-8 of the whole gradient's norm), not equal noise
    gn = float(g0.double().norm())
    floor = 1e-6 * gn
    for name, view in st.P.named.items():
        o = view.storage_offset() - st.flat.storage_offset()
        a, b = g1[o:o + view.numel()].double(), g0[o:o + view.numel()].double()
        if o == o_w or o == o_b:
            continue
        if name.endswith("lin_key.bias"):
            assert float(a.norm()) < 1e-8 * gn and float(b.norm()) < 1e-8 * gn, name
            continue
        assert float((a - b).norm()) / max(float(b.norm()), floor) < 1e-5, name
