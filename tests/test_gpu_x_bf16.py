"""bf16 GEMM arithmetic (ALIGNN_GEMM_BF16; SURVEY §8d config C3 — the reference's CUDA autocast
GEMMs, train.py:632-636): inputs rounded to bf16 (RNE) into v_mfma_f32_32x32x16_bf16, fp32
accumulation and storage.  The exact reference for that arithmetic is an fp64 product of the
bf16-rounded operands (bf16 x bf16 products are exact in fp32, so only the fp32 summation order
differs): tolerance 5e-6 relative to the largest output.  Engine level: a bf16 training step against
the fp32 one (loss within 2e-2 relative, gradient cosine > 0.999).  Sorts after the core suites."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30))


def _rb(x):
    return x.bfloat16().double()


@pytest.mark.parametrize("tile", [0, 1, 2, 3, 4, 17, 20])
@pytest.mark.parametrize("layout", ["nt", "nn", "tn", "tt"])
def test_gemm_bf16_layouts_and_tiles(tile, layout):
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(tile * 5 + len(layout) + ord(layout[0]))
    M, N, K = 300, 257, 1000
    A = torch.randn(M, K, generator=g).to(DEV)
    B = torch.randn(K, N, generator=g).to(DEV)
    Av = A if layout[0] == "n" else A.t().contiguous().t()
    Bv = B if layout[1] == "n" else B.t().contiguous().t()
    ref = _rb(A) @ _rb(B)
    for split in (1, 3):
        C = torch.empty(M, N, device=DEV)
        ops.gemm(Av, Bv, C, tile=tile | ops.GEMM_BF16, split_k=split)
        assert _rel(C, ref) < 5e-6, (split,)
    # the flag is really applied: the bf16 result is NOT the fp32 product
    assert _rel(C, A.double() @ B.double()) > 1e-4


def test_gemm_bf16_context_epilogue_reduce_batch_and_scatter():
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(3)
    M, N, K = 200, 96, 48
    A = torch.randn(M, K, generator=g).to(DEV)
    W = torch.randn(N, K, generator=g).to(DEV)
    bias = torch.randn(N, generator=g).to(DEV)
    C = torch.randn(M, N, generator=g).to(DEV)
    C0 = C.clone()
    with ops.gemm_precision("bf16"):
        ops.gemm(A, W.t(), C, beta=0.5, bias=bias, relu=True)
    ref = torch.relu(_rb(A) @ _rb(W).t() + 0.5 * C0.double() + bias.double())
    assert _rel(C, ref) < 5e-6
    # context restored: fp32 again afterwards
    C2 = torch.empty(M, N, device=DEV)
    ops.gemm(A, W.t(), C2)
    assert _rel(C2, A.double() @ W.double().t()) < 2e-6
    # batch-reduced weight gradient (shared angle projection) in bf16
    Ab = torch.randn(4, 64, 256, generator=g).to(DEV)
    Bb = torch.randn(4, 256, 96, generator=g).to(DEV)
    Cb = torch.empty(64, 96, device=DEV)
    with ops.gemm_precision("bf16"):
        ops.gemm(Ab, Bb, Cb, reduce_batch=True)
    assert _rel(Cb, (_rb(Ab) @ _rb(Bb)).sum(0)) < 5e-6
    # row scatter
    rows = torch.randperm(300, generator=g)[:M].to(torch.int32).to(DEV)
    Cs = torch.zeros(300, N, device=DEV)
    with ops.gemm_precision("bf16"):
        ops.gemm(A, W.t(), Cs, c_rows=rows)
    assert _rel(Cs[rows.long()], _rb(A) @ _rb(W).t()) < 5e-6
    with pytest.raises(ValueError):
        with ops.gemm_precision("fp16"):
            pass


def test_bf16_training_step_tracks_fp32():
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    res = {}
    for prec in ("fp32", "bf16"):
        torch.manual_seed(0)
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(DEV)
        tr = A.FusedTrainer(model, precision=prec)
        assert model._engine.precision == prec
        b = mp_like_batch(4).to(DEV)
        loss = tr.forward_backward(b, 5, training=False).clone()
        torch.cuda.synchronize()
        res[prec] = (loss, tr.st.grad.clone())
    (l32, g32), (l16, g16) = res["fp32"], res["bf16"]
    assert torch.isfinite(l16).all() and torch.isfinite(g16).all()
    assert abs(float(l16) - float(l32)) <= 2e-2 * abs(float(l32))
    cos = float((g16.double() @ g32.double()) / (g16.double().norm() * g32.double().norm()))
    assert cos > 0.999, cos
    assert not torch.equal(g16, g32)   # bf16 arithmetic really used


def test_bf16_storage_attention_vs_fp32_kernels_on_rounded_inputs():
    """alignn_lg_fwd_bf16 / alignn_lg_bwd_dst_bf16 widen bf16 rows exactly, so on K|V and F rows that
    are bf16-representable they compute what the fp32 single-wave-item kernels compute, with dropout
    on; ragged in-degrees incl. 0 and group tails.  They run one edge group in flight (the fp32
    kernels two), and the compiler contracts their per-edge softmax terms differently between the
    two (measured: 1-ulp differences, tools/lg_diff.py), so the outputs are held to fp32 rounding
    (1e-5 of each output's largest magnitude) rather than bits."""
    from alignn_mi355x import ops
    from test_gpu_x_lg3 import DEGREES, _case
    for H in (1, 2, 4):
        for drop in (0.0, 0.15):
            csr, m, t = _case(H, DEGREES["ragged"] + DEGREES["mp_mix"][:20], 90 + H, True)
            n, D = csr.n, 256
            QKV = t["QKVR"][:, :3 * D].contiguous()
            QKV[:, D:3 * D] = QKV[:, D:3 * D].bfloat16().float()     # K|V representable in bf16
            F = t["F"].bfloat16().float()
            KV16 = ops.cast_bf16(QKV[:, D:3 * D])
            F16 = ops.cast_bf16(F)
            outs = {}
            for mode in ("fp32", "bf16"):
                outp, S = torch.empty(n, D, device=DEV), torch.empty(n, H, D, device=DEV)
                sumA, mstat, den = (torch.empty(n, H, device=DEV) for _ in range(3))
                dq = torch.empty(n, D, device=DEV)
                Sz, sigz = torch.empty(n, H, D, device=DEV), torch.empty(n, H, device=DEV)
                dz, al = torch.empty(max(m, 1), H, device=DEV), torch.empty(max(m, 1), H, device=DEV)
                if mode == "fp32":
                    assert csr.family(D, H, F) == 3
                    ops.tconv_fwd(csr, D, H, QKV, t["U"], t["wbar"], F, None, outp, S, sumA, mstat, den, drop, 5)
                    ops.tconv_bwd_dst(csr, D, H, QKV, t["U"], t["Vd"], t["wbar"], F, None, t["dout"], outp, mstat,
                                      den, dq, Sz, sigz, dz, al, None, 0, drop, 5)
                else:
                    ops.lg_fwd_bf16(csr, D, H, QKV, KV16, t["U"], t["wbar"], F16, outp, S, sumA, mstat, den, drop, 5)
                    ops.lg_bwd_dst_bf16(csr, D, H, QKV, KV16, t["U"], t["Vd"], t["wbar"], F16, t["dout"], outp,
                                        mstat, den, dq, Sz, sigz, dz, al, drop, 5)
                torch.cuda.synchronize()
                outs[mode] = dict(outp=outp, S=S, sumA=sumA, mstat=mstat, den=den, dq=dq, Sz=Sz, sigz=sigz,
                                  dz=dz[:m], al=al[:m])
            for k in outs["fp32"]:
                a, r = outs["bf16"][k].double(), outs["fp32"][k].double()
                fin = torch.isfinite(r)   # mstat is -inf on targets without in-edges
                assert torch.equal(torch.isfinite(a), fin) and torch.equal(a[~fin], r[~fin]), (k, H, drop)
                a, r = a[fin], r[fin]
                if r.numel():
                    assert float((a - r).abs().max()) <= 1e-5 * max(float(r.abs().max()), 1e-30), (k, H, drop)


def test_cast_and_skinny_bf16_outputs_bitwise():
    """alignn_cast_bf16_f32 rounds to nearest even exactly like torch's fp32 -> bf16 conversion;
    alignn_linear_smallk_bf16out is the Linear + ReLU as bf16 autocast computes it (train.py:554 under
    :636): bf16 x, W, b, exact products summed in fp32, the sum rounded to bf16 — against the float64 sum
    of the same bf16 operands rounded once, every element within one bf16 rounding step and all but a
    few (sums within fp32 error of a rounding boundary) equal."""
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(12)
    x = (torch.randn(1037, 260, generator=g) * 3).to(DEV)
    x[0, :4] = torch.tensor([1.0 + 2 ** -8, 1.0 + 3 * 2 ** -8, -0.0, 65504.0])  # ties round to even
    assert torch.equal(ops.cast_bf16(x), x.bfloat16())
    xs = x[:, 4:260]                                                           # strided source rows
    assert torch.equal(ops.cast_bf16(xs), xs.bfloat16())
    X = torch.randn(5000, 11, generator=g).to(DEV)
    W = torch.randn(256, 11, generator=g).to(DEV)
    b = torch.randn(256, generator=g).to(DEV)
    h16 = torch.empty(5000, 256, device=DEV, dtype=torch.bfloat16)
    ops.linear_smallk_bf16(X, W, b, h16, relu=True)
    bf = lambda t: t.bfloat16().double()  # noqa: E731
    ref = torch.relu((bf(X) @ bf(W).t() + bf(b)).float().bfloat16().float())
    got = h16.float()
    assert torch.equal(got > 0, ref > 0) or float(((got > 0) != (ref > 0)).float().mean()) < 1e-5
    ulp = ref.abs().clamp_min(2.0 ** -126) * 2.0 ** -7
    assert bool(((got - ref).abs() <= ulp).all())
    assert float((got != ref).float().mean()) < 1e-3
    # rows past a 32-row chunk, and a bias-free call
    h = torch.full((37, 256), 7.0, device=DEV, dtype=torch.bfloat16)
    ops.linear_smallk_bf16(X[:37], W, None, h, relu=False)
    ref = (bf(X[:37]) @ bf(W).t()).float()
    assert float(((h.float() - ref).abs() / ref.abs().clamp_min(1e-3)).max()) < 1e-2


def test_bf16_storage_step_vs_float64_oracle():
    """The config-C3 precision policy end to end (bf16 GEMM inputs, bf16 angle hidden layer and K|V
    rows in the line-graph attention, fp32 everything else) against the float64 oracle of the
    reference's step on a B = 4 MP-like batch (dropout 0, jitter 0).  Stated bf16 tolerance: loss
    within 1e-2 relative, cosine of the flat gradient > 0.999, per-parameter normwise error below
    max(5e-2, 2 x the error of the bf16-GEMM-only step) for every parameter with a gradient norm
    above 1e-3 of the largest — the gate weights lin_beta.weight are ill-conditioned sums (large
    cancelling terms; even the reference's fp32 CPU path misses fp64 by 1.7e-4 there at B = 32,
    test_gpu_parity.py), so their bf16 error is bounded by the bf16 GEMM path's own.  The storage
    path is really taken: its gradient differs from the bf16-GEMM-only step."""
    import alignn_mi355x as A
    from alignn_mi355x.layout import offsets
    from alignn_mi355x.synthetic import mp_like_batch
    from oracle import model_ref
    from oracle.pyg_ref import RefData
    torch.manual_seed(3)
    proto = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.0), 2)
    st = {k: v.detach().clone() for k, v in proto.state_dict().items()}
    cpu_b = mp_like_batch(4)
    ref_b = RefData(**{k: getattr(cpu_b, k) for k in cpu_b.keys()})
    for k in ("x", "edge_attr", "lg_edge_attr", "global_x", "sg_one_hot", "y"):
        setattr(ref_b, k, getattr(ref_b, k).double())
    ref_b.num_graphs = 4
    ps = {k: v.double().requires_grad_(True) for k, v in st.items()}
    mean, logvar = model_ref.hetero_forward(ps, ref_b, 4)
    tz = model_ref.log_transform(ref_b.y.view(4, -1), (4.3228, 3.5567), (0.9051, 0.9405))
    rloss = model_ref.hetero_loss(mean, logvar, tz, 0.1)
    rloss.backward()
    res = {}
    for storage in (True, False):
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.0), 2)
        model.load_state_dict(st)
        model.to(DEV)
        model._engine.bf16_storage = storage
        tr = A.FusedTrainer(model, precision="bf16", feature_jitter_std=0.0, target_log_means=(4.3228, 3.5567),
                            target_log_stds=(0.9051, 0.9405))
        loss = tr.forward_backward(cpu_b.to(DEV), 5).clone()
        torch.cuda.synchronize()
        res[storage] = (loss, tr.st.grad.clone(), model)
    l16, g16, model = res[True]
    assert not torch.equal(g16, res[False][1])
    assert abs(float(l16) - float(rloss)) <= 1e-2 * abs(float(rloss))
    offs, _, _ = offsets(model.config, True)
    gref = torch.zeros_like(g16, dtype=torch.float64, device="cpu")
    for k, (o, shape) in offs.items():
        if ps[k].grad is not None:
            gref[o:o + ps[k].numel()] = ps[k].grad.reshape(-1)
    g = g16.double().cpu()
    g0 = res[False][1].double().cpu()
    assert float(g @ gref / (g.norm() * gref.norm())) > 0.999
    top = max(float(p.grad.norm()) for p in ps.values() if p.grad is not None)
    for k, (o, shape) in offs.items():
        if ps[k].grad is None or float(ps[k].grad.norm()) < 1e-3 * top:
            continue
        ga, gz, gb = g[o:o + ps[k].numel()], g0[o:o + ps[k].numel()], gref[o:o + ps[k].numel()]
        err, err_gemm = float((ga - gb).norm() / gb.norm()), float((gz - gb).norm() / gb.norm())
        assert err < max(5e-2, 2.0 * err_gemm), (k, err, err_gemm)
