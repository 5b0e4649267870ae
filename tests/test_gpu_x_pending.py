"""GPU tests of engine options and kernel variants: GEMM stage depths, stream-placement options
(bitwise neutral), the HIP optimizer, tconv.hip's light/heavy attention kernels vs fp64.  Kept in a file that sorts
after the core parity suites so a failure here cannot stop those under ``pytest -x``."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ops():
    from alignn_mi355x import ops
    return ops


def _rel(a, b):
    """Max-abs difference relative to max |b|; equal entries (incl. matching -inf softmax maxima
    of zero in-degree targets) count as 0."""
    a, b = a.double(), b.double()
    d = torch.where(a == b, torch.zeros_like(a), a - b)
    fin = b[torch.isfinite(b)]
    return float(d.abs().max() / (fin.abs().max() if fin.numel() else torch.tensor(1.0)).clamp(min=1e-30))


def _setup(seed=0):
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    torch.manual_seed(seed)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(DEV)
    tr = A.FusedTrainer(model)
    b = mp_like_batch(4).to(DEV)
    return model, tr, b


@pytest.mark.parametrize("stage", [16, 128])
@pytest.mark.parametrize("shape", [1, 2, 3, 4])
@pytest.mark.parametrize("layout", ["nt", "nn", "tn", "tt"])
def test_gemm_bk32_stage(shape, layout, stage):
    """32-deep (ALIGNN_GEMM_BK32 = 16) and 64-deep (ALIGNN_GEMM_BK64 = 128) K stages on every tile
    shape and operand layout, unsplit and split-K (K = 1000: a partial last stage)."""
    ops = _ops()
    g = torch.Generator(device="cpu").manual_seed(shape * 11 + len(layout))
    M, N, K = 300, 257, 1000
    A = torch.randn(M, K, generator=g).to(DEV)
    B = torch.randn(K, N, generator=g).to(DEV)
    Av = A if layout[0] == "n" else A.t().contiguous().t()
    Bv = B if layout[1] == "n" else B.t().contiguous().t()
    ref = A.double() @ B.double()
    for split in (1, 3):
        C = torch.empty(M, N, device=DEV)
        ops.gemm(Av, Bv, C, tile=stage + shape, split_k=split)
        assert _rel(C, ref) < 5e-6, (split,)
    # batch-reduced (shared weights): K multiple of 32 keeps the 32-deep stage inside one batch entry
    Ab = torch.randn(4, 64, 256, generator=g).to(DEV)
    Bb = torch.randn(4, 256, 96, generator=g).to(DEV)
    Cb = torch.empty(64, 96, device=DEV)
    ops.gemm(Ab, Bb, Cb, reduce_batch=True, tile=stage + shape)
    assert _rel(Cb, (Ab.double() @ Bb.double()).sum(0)) < 5e-6



def test_forward_side_stream_is_bitwise_neutral():
    """The line blocks' skip projection on the side stream (overlap_forward) changes no bits."""
    _, tr1, b1 = _setup()
    _, tr2, b2 = _setup()
    tr1.model._engine.overlap_forward = False
    tr2.model._engine.overlap_forward = True
    l1 = tr1.forward_backward(b1, 9)
    l2 = tr2.forward_backward(b2, 9)
    torch.cuda.synchronize()
    assert torch.equal(l1, l2)
    assert torch.equal(tr1.st.grad, tr2.st.grad)


@pytest.mark.parametrize("flag,value", [("enc_bwd_aux", 1), ("gate_reduce_side", True), ("wgrad_early", 1),
                                        ("wgrad_early", 2)])
def test_backward_third_stream_is_bitwise_neutral(flag, value):
    """Branches off the main stream (the deferred angle-encoder backward on the third stream, the
    gate/LayerNorm parameter reduction on the side stream, the weight gradients queued before dX)
    change no bits."""
    _, tr1, b1 = _setup()
    _, tr2, b2 = _setup()
    setattr(tr1.model._engine, flag, type(value)(0))
    setattr(tr2.model._engine, flag, value)
    l1 = tr1.forward_backward(b1, 9)
    l2 = tr2.forward_backward(b2, 9)
    torch.cuda.synchronize()
    assert torch.equal(l1, l2)
    assert torch.equal(tr1.st.grad, tr2.st.grad)


def test_hip_clip_adamw_matches_torch():
    """alignn_grad_norm_f32 + alignn_adamw_f32 vs torch clip_grad_norm_ + the single-tensor AdamW (the
    reference's CPU optimizer, train.py:1537-1540 without fused=True), 3 steps, two param groups with
    different learning rates.  (torch's fused GPU AdamW rounds 1 - beta2 from the fp32 beta2, 1.3e-5
    away from the CPU path's 0.001f, so it is not the reference here.)"""
    ops = _ops()
    torch.manual_seed(4)
    n, split = 100_003, 90_001
    p0 = torch.randn(n, device=DEV)
    pa = torch.nn.Parameter(p0[:split].clone())
    pb = torch.nn.Parameter(p0[split:].clone())
    opt = torch.optim.AdamW([{"params": [pa], "lr": 3e-4}, {"params": [pb], "lr": 1e-4}], lr=3e-4,
                            weight_decay=1e-4, foreach=False, fused=False)
    p = p0.clone()
    m = torch.zeros(n, device=DEV)
    v = torch.zeros(n, device=DEV)
    step = torch.zeros(1, device=DEV)
    norm = torch.zeros(1, device=DEV)
    for it in range(3):
        g = torch.randn(n, device=DEV) * (4.0 if it == 0 else 0.01)   # first step clips, later ones do not
        pa.grad, pb.grad = g[:split].clone(), g[split:].clone()
        torch.nn.utils.clip_grad_norm_([pa, pb], max_norm=5.0)
        opt.step()
        gg = g.clone()
        ops.grad_norm(gg, norm)
        assert abs(float(norm) - float(g.double().norm())) < 1e-5 * float(g.double().norm())
        ops.adamw_step(p, gg, m, v, split, 3e-4, 1e-4, 1e-4, norm=norm, max_norm=5.0, step=step)
        assert _rel(gg, torch.cat([pa.grad, pb.grad])) < 1e-6, it
        # parameters: both sides round p in fp32, so allow 2 ulp of |p| on top of 1e-4 of the update
        pt = torch.cat([pa.detach(), pb.detach()])
        tol = 1e-4 * (pt - p0).abs().max() + 2 * torch.finfo(torch.float32).eps * p.abs()
        assert bool(((p - pt).abs() <= tol).all()), (it, float((p - pt).abs().max()))
        mt = torch.cat([opt.state[pa]["exp_avg"], opt.state[pb]["exp_avg"]])
        vt = torch.cat([opt.state[pa]["exp_avg_sq"], opt.state[pb]["exp_avg_sq"]])
        assert _rel(m, mt) < 1e-5 and _rel(v, vt) < 1e-5, it
    assert float(step) == 3.0


def test_fused_trainer_hip_optimizer_vs_reference_golden(golden):
    """One full training step with the HIP clip + AdamW vs the reference's train_epoch_hetero."""
    import alignn_mi355x as A
    from _golden_util import batch_from, meta, rel_err, state_from
    g = golden("mp_d64_quirk")
    mt = meta(g)
    base = A.AlignnRegressor(int(mt["node"]), int(mt["edge"]), int(mt["angle"]), int(mt["global"]), 2,
                             int(mt["hidden"]), int(mt["layers"]), int(mt["heads"]), 0.0)
    model = A.HeteroAlignnRegressor(base, 2)
    model.load_state_dict(state_from(g, dtype=torch.float32))
    model.to(DEV).train()
    b = batch_from(g, A.Batch, torch.float32).to(DEV)
    tr = A.FusedTrainer(model, feature_jitter_std=0.0, target_log_means=mt["target_means"],
                        target_log_stds=mt["target_stds"], optimizer="hip")
    tr.step(b, seed=0)
    for k, v in model.state_dict().items():
        if k.endswith("lin_key.bias"):
            continue
        assert rel_err(v.cpu(), g[f"f32/post/{k}"]) < 1e-4, k


def test_hetero_nll_with_knn_sample_weights():
    """Weighted NLL (train.py:660-674: nll * w per graph, L2 term unweighted) vs torch fp64 autograd."""
    ops = _ops()
    torch.manual_seed(8)
    B, T = 16, 2
    heads = torch.randn(B, 2 * T, device=DEV)
    y = torch.rand(B * T, device=DEV) * 299 + 1
    w = torch.rand(B, device=DEV) * 2
    lm = torch.tensor([4.3228, 3.5567], device=DEV)
    ls = torch.tensor([0.9051, 0.9405], device=DEV)
    loss = torch.zeros(1, device=DEV)
    dh = torch.empty_like(heads)
    ops.hetero_nll(heads, y, lm, ls, -2.9, 0.1, loss, dh, weights=w)
    h = heads.double().clone().requires_grad_(True)
    mean, logvar = h[:, :T], h[:, T:]
    tz = (torch.log(y.double().view(B, T)) - lm.double()) / ls.double()
    lv = torch.clamp(logvar, min=-2.9)
    nll = 0.5 * (lv + (mean - tz) ** 2 / torch.exp(lv)) * w.double().view(-1, 1)
    ref = nll.mean(1).mean() + 0.1 * (0.5 * lv).pow(2).mean()
    ref.backward()
    assert abs(float(loss) - float(ref)) < 1e-5 * abs(float(ref))
    assert _rel(dh, h.grad) < 1e-5


def _tconv_case(D, H, n, deg_hi, seed, with_wbar, feat_row):
    """Random graph with ragged in-degrees (some 0, some above the heavy threshold) and operands."""
    ops = _ops()
    g = torch.Generator().manual_seed(seed)
    degs = torch.randint(0, deg_hi, (n,), generator=g)
    degs[::7] = 0
    dst = torch.repeat_interleave(torch.arange(n), degs)
    src = torch.randint(0, n, (dst.numel(),), generator=g)
    ei = torch.stack([src, dst]).to(DEV)
    csr = ops.GraphCSR(ei, n)
    m = dst.numel()
    r = lambda *s: (torch.randn(*s, generator=g) * 0.5).to(DEV)  # noqa: E731
    t = dict(QKVR=r(n, 4 * D), U=r(n, H, D), Vd=r(n, H, D), F=r(max(m, 1), D), dout=r(n, D),
             wbar=r(D) if with_wbar else None, dF0=r(max(m, 1), D),
             feat_row=(torch.randperm(max(m, 1), generator=g)[:m].to(torch.int32).to(DEV) if feat_row else None))
    return csr, m, t


def _run_tconv(csr, m, t, D, H, drop, heavy_threshold):
    """tconv.hip's light/heavy kernels (wave_items off: every shape takes them, D = 256 included)."""
    ops = _ops()
    n = csr.n
    csr._sched = None
    csr.policy = ops.SchedulePolicy(heavy_threshold=heavy_threshold, wave_items=False)
    assert csr.family(D, H, t["F"], t["feat_row"]) == 2
    outp, S = torch.empty(n, D, device=DEV), torch.empty(n, H, D, device=DEV)
    sumA, mstat, den = (torch.empty(n, H, device=DEV) for _ in range(3))
    ops.tconv_fwd(csr, D, H, t["QKVR"], t["U"], t["wbar"], t["F"], t["feat_row"], outp, S, sumA, mstat, den,
                  drop, 77)
    dq = torch.empty(n, D, device=DEV)
    Sz, sigz = torch.empty(n, H, D, device=DEV), torch.empty(n, H, device=DEV)
    dz, al = torch.empty(max(m, 1), H, device=DEV), torch.empty(max(m, 1), H, device=DEV)
    dF = t["dF0"].clone()
    ops.tconv_bwd_dst(csr, D, H, t["QKVR"], t["U"], t["Vd"], t["wbar"], t["F"], t["feat_row"], t["dout"], outp,
                      mstat, den, dq, Sz, sigz, dz, al, dF, 3, drop, 77)
    torch.cuda.synchronize()
    return dict(outp=outp, S=S, sumA=sumA, mstat=mstat, den=den, dq=dq, Sz=Sz, sigz=sigz, dz=dz[:m], al=al[:m],
                dF=dF)


def _attention_ref(csr, m, t, D, H):
    """fp64 restatement of the kernels' contract (include/alignn_hip.h, alignn_tconv_fwd/_bwd_dst;
    PyG TransformerConv.message + softmax(+1e-16) with the edge-feature algebra of DESIGN.md §3),
    no dropout.  Edge position t: target-sorted (csr.src_at / dst_at); F row feat_row[t] or t."""
    import math
    n, C = csr.n, D // H
    d64 = lambda x: x.detach().double().cpu()  # noqa: E731
    src, dst = csr.src_at[:m].long().cpu(), csr.dst_at[:m].long().cpu()
    row = t["feat_row"][:m].long().cpu() if t["feat_row"] is not None else torch.arange(m)
    QKVR = d64(t["QKVR"])
    Q, K, V = (QKVR[:, i * D:(i + 1) * D].reshape(n, H, C) for i in range(3))
    U, Vd, F = d64(t["U"]), d64(t["Vd"]), d64(t["F"])[row]
    wb = d64(t["wbar"]).view(H, C) if t["wbar"] is not None else torch.zeros(H, C, dtype=torch.float64)
    dout = d64(t["dout"]).view(n, H, C)
    z64 = lambda *s: torch.zeros(*s, dtype=torch.float64)  # noqa: E731
    z = ((Q[dst] * K[src]).sum(-1) + torch.einsum("mhd,md->mh", U[dst], F) + (Q[dst] * wb).sum(-1)) / math.sqrt(C)
    mst = torch.full((n, H), float("-inf"), dtype=torch.float64).scatter_reduce(
        0, dst[:, None].expand(m, H), z, "amax", include_self=True)
    ex = torch.exp(z - mst[dst])
    den = z64(n, H).index_add_(0, dst, ex) + 1e-16
    al = ex / den[dst]
    outp = z64(n, H, C).index_add_(0, dst, al[..., None] * V[src]).view(n, D)
    S = z64(n, H, D).index_add_(0, dst, al[..., None] * F[:, None, :])
    sumA = z64(n, H).index_add_(0, dst, al)
    g = (dout[dst] * V[src]).sum(-1) + torch.einsum("mhd,md->mh", Vd[dst], F) + (dout[dst] * wb).sum(-1)
    pdl = (dout * outp.view(n, H, C)).sum(-1)
    dz = al * (g - pdl[dst]) / math.sqrt(C)
    dq = z64(n, H, C).index_add_(0, dst, dz[..., None] * K[src]).view(n, D)
    Sz = z64(n, H, D).index_add_(0, dst, dz[..., None] * F[:, None, :])
    sigz = z64(n, H).index_add_(0, dst, dz)
    dF = d64(t["dF0"])
    upd = torch.einsum("mh,mhd->md", dz, U[dst]) + torch.einsum("mh,mhd->md", al, Vd[dst])
    dF[row] = (dF[row] + upd) * (F > 0)            # accumulate_dF = 3: add, then the ReLU mask
    return dict(outp=outp, S=S, sumA=sumA, mstat=mst, den=den, dq=dq, Sz=Sz, sigz=sigz, dz=dz, al=al, dF=dF)


@pytest.mark.parametrize("thr", [32, 256])
@pytest.mark.parametrize("D,H", [(256, 4), (128, 2), (64, 1), (32, 4), (32, 1), (512, 8)])
def test_light_heavy_attention_kernels_vs_fp64(D, H, thr):
    """tconv.hip's attention kernels (forward + target-side backward with the dF read-modify-write
    path, every supported D/H) vs an fp64 restatement of their contract: 2e-5 of each output's max.
    thr: heavy-node threshold (32: in-degrees up to 70 take both the 4-wave and the 1-wave path;
    256, the default: all 1-wave)."""
    for seed, (with_wbar, feat_row) in enumerate([(True, False), (False, True)]):
        csr, m, t = _tconv_case(D, H, 300, 70, 10 + seed, with_wbar, feat_row)
        got = _run_tconv(csr, m, t, D, H, 0.0, thr)
        ref = _attention_ref(csr, m, t, D, H)
        for k in ref:
            assert _rel(got[k].cpu(), ref[k]) < 2e-5, (k, D, H, thr, seed)


@pytest.mark.parametrize("D,H", [(256, 4), (128, 2)])
def test_light_heavy_attention_dropout_replays(D, H):
    """With dropout the kernels draw the same keep mask in the forward and the backward (the alpha'
    they write per edge sums to sumA), and a second run is bitwise identical."""
    csr, m, t = _tconv_case(D, H, 300, 70, 21, True, False)
    a = _run_tconv(csr, m, t, D, H, 0.15, 32)
    b = _run_tconv(csr, m, t, D, H, 0.15, 32)
    for k in a:
        assert torch.equal(a[k], b[k]), k
    dst = csr.dst_at[:m].long()
    sumA = torch.zeros(csr.n, H, device=DEV, dtype=torch.float64).index_add_(0, dst, a["al"].double())
    assert _rel(a["sumA"], sumA) < 1e-5
    assert float((a["al"] == 0).double().mean()) > 0.1     # ~15 % of (edge, head) pairs dropped


@pytest.mark.parametrize("lg_offset", ["num_nodes", "num_edges"])
def test_light_heavy_kernels_full_model_vs_oracle(lg_offset, monkeypatch):
    """The production model (D = 256) with every attention on tconv.hip's kernels (wave_items off)
    vs the fp64 oracle."""
    import alignn_mi355x as A
    from alignn_mi355x import ops
    from alignn_mi355x.synthetic import mp_like_batch
    from oracle import model_ref
    from oracle.pyg_ref import RefData
    monkeypatch.setattr(ops, "DEFAULT_SCHEDULE", ops.SchedulePolicy(wave_items=False))
    torch.manual_seed(5)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.0), 2)
    st = {k: v.detach().clone().double() for k, v in model.state_dict().items()}
    cpu_batch = mp_like_batch(3, lg_offset=lg_offset)
    ref_b = RefData(**{k: getattr(cpu_batch, k) for k in cpu_batch.keys()})
    for k in ("x", "edge_attr", "lg_edge_attr", "global_x", "sg_one_hot", "y"):
        setattr(ref_b, k, getattr(ref_b, k).double())
    ref_b.num_graphs = 3
    rmean, rlogvar = model_ref.hetero_forward(st, ref_b, 4)
    model.to(DEV)
    b = cpu_batch.to(DEV)
    mean, logvar = model(b)
    assert b._alignn_cache.lg.policy.wave_items is False
    assert _rel(mean.detach().cpu(), rmean) < 1e-4
    assert _rel(logvar.detach().cpu(), rlogvar) < 1e-4


def test_atom_blocks_on_aux_stream():
    """atom_stream: the atom-graph blocks' edge-feature gradient in a buffer of its own (1) equals
    the in-kernel accumulation (0) to fp32 rounding (one add instead of a fused chain), and running
    the atom blocks on the aux stream beside the line blocks (2) changes no bits against 1 — eager
    and as a captured plan."""
    _, tr0, b0 = _setup()
    _, tr1, b1 = _setup()
    _, tr2, b2 = _setup()
    tr0.model._engine.atom_stream = 0
    tr1.model._engine.atom_stream = 1
    tr2.model._engine.atom_stream = 2
    l0 = tr0.forward_backward(b0, 9)
    l1 = tr1.forward_backward(b1, 9)
    l2 = tr2.forward_backward(b2, 9)
    torch.cuda.synchronize()
    assert torch.equal(l1, l2)
    assert torch.equal(tr1.st.grad, tr2.st.grad)
    assert torch.equal(l0, l1)   # the forward is untouched
    g0, g1 = tr0.st.grad.double(), tr1.st.grad.double()
    assert float((g0 - g1).norm() / g0.norm()) < 1e-5
    # captured (mode 2, plan replay) against eager steps of the mode-1 twin, same device step seed
    from alignn_mi355x import ops
    _, tr3, b3 = _setup()
    _, tr4, b4 = _setup()
    tr3.model._engine.atom_stream = 1
    tr4.model._engine.atom_stream = 2
    tr4.capture(b4, mode="plan")
    for i, s in enumerate((11, 12, 13)):
        tr3.use_step_seed(tr4._seed_dev)
        tr4._seed_dev.fill_(s)
        l3 = tr3.forward_backward(b3, 0).clone()
        tr3._clip_and_update()
        l4 = tr4.step(b4, seed=s).clone()
        torch.cuda.synchronize()
        assert torch.equal(l3, l4), i
        assert torch.equal(tr3.st.flat, tr4.st.flat), i
    ops.set_step_seed(None)
