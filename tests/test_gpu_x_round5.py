"""Round-5 GPU checks: the drop-in module under the reference's own CUDA autocast (train.py:632-636,
:653-681, :690-695).

* ``alignn_hetero_nll_amp`` against torch's autograd of the reference's loss lines under
  ``torch.autocast("cuda", bfloat16)`` on the same bf16 heads: gradients bit for bit, loss to fp32
  summation order.
* A restatement of ``train_epoch_hetero``'s amp branch (autocast + ``torch.amp.GradScaler`` +
  ``clip_grad_norm_`` + AdamW) through the module API against ``FusedTrainer(precision="bf16")``:
  heads bitwise, every parameter gradient bitwise, the post-step parameters to the optimizer
  tolerance of test_hip_clip_adamw_matches_torch (torch's AdamW vs the library's), and a skipped
  (non-finite) step skipped by both with the same scale back-off.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
FLOOR = -2.9          # MIN_LOGVAR_FLOOR (train.py)
LOG_MEANS = (4.3228, 3.5567)   # alignn_mi355x.synthetic.TARGET_LOG_* (the trainer's LogTransformer state)
LOG_STDS = (0.9051, 0.9405)


def _ref_loss(mean, logvar, y, lm, ls, l2, w=None):
    """train.py:648-681 (with transformer.transform_tensor, train.py:268-279), as written; the caller
    holds the autocast context."""
    target_trans = (torch.log(y) - lm) / ls
    logvar = torch.clamp(logvar, min=FLOOR)
    logvar_loss = logvar
    var = torch.exp(logvar_loss)
    diff = mean - target_trans.to(mean.dtype)
    nll = 0.5 * (logvar_loss + diff.pow(2) / var)
    if w is not None:
        nll = nll * w.view(-1, 1)
    sample_loss = nll.mean(dim=1)
    loss = sample_loss.mean()
    if l2 > 0.0:
        log_sigma = 0.5 * logvar_loss
        loss = loss + float(l2) * log_sigma.pow(2).mean()
    return loss


@pytest.mark.parametrize("weighted", [False, True])
@pytest.mark.parametrize("B", [32, 7, 256])
def test_amp_loss_kernel_matches_autocast_autograd(weighted, B):
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(B + weighted)
    T = 2
    heads = (torch.randn(B, 2 * T, generator=g) * 2.0).to(DEV)
    heads[0, T] = -7.0                         # below the floor: clamp's zero gradient
    heads[1, T + 1] = -2.9                     # rounds to the bf16 floor itself (subgradient 1)
    y = (torch.rand(B, T, generator=g) * 299 + 1).to(DEV)
    w = (torch.rand(B, generator=g) + 0.5).to(DEV) if weighted else None
    lm = torch.tensor(LOG_MEANS, device=DEV)
    ls = torch.tensor(LOG_STDS, device=DEV)
    S = 65536.0
    h16 = heads.to(torch.bfloat16).requires_grad_(True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        loss = _ref_loss(h16[:, :T], h16[:, T:], y, lm, ls, 0.1, w)
    (loss * torch.tensor(S, device=DEV)).backward()
    ref = h16.grad.float() / S
    out_loss = torch.zeros(1, device=DEV)
    dh = torch.empty_like(heads)
    ops.hetero_nll(heads, y, lm, ls, FLOOR, 0.1, out_loss, dh, weights=w, amp=True)
    torch.cuda.synchronize()
    assert torch.equal(dh, ref), float((dh - ref).abs().max())
    assert abs(float(out_loss) - float(loss)) <= 2e-6 * abs(float(loss))


def _model(seed, dropout=0.15):
    import alignn_mi355x as A
    torch.manual_seed(seed)
    return A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, dropout), 2).to(DEV)


def _reference_amp_step(model, opt, scaler, batch, draw_seed):
    """One iteration of train_epoch_hetero's loop body with use_amp (train.py:647-699), jitter off."""
    opt.zero_grad(set_to_none=True)
    target = batch.y.view(batch.num_graphs, -1)
    lm = torch.tensor(LOG_MEANS, device=DEV)
    ls = torch.tensor(LOG_STDS, device=DEV)
    torch.manual_seed(draw_seed)                 # the module draws its dropout seed from torch's generator
    with torch.autocast(device_type="cuda", dtype=torch.bfloat16):
        mean, logvar = model(batch)
        heads = torch.cat([mean, logvar], 1).detach().clone()
        loss = _ref_loss(mean, logvar, target, lm, ls, 0.1)
    scaler.scale(loss).backward()
    scaler.unscale_(opt)
    grads = {k: p.grad.detach().clone() for k, p in model.named_parameters() if p.grad is not None}
    norm = torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=5.0)
    scaler.step(opt)
    scaler.update()
    return loss.detach(), heads, grads, float(norm)


def _torch_adamw(model):
    """The reference's two parameter groups (train.py:1516-1542) on torch's single-tensor AdamW (the
    arithmetic the library's optimizer restates)."""
    base = list(model.base.parameters()) + list(model.mean_heads.parameters())
    sigma = list(model.logvar_heads.parameters())
    return torch.optim.AdamW([{"params": base, "lr": 3e-4}, {"params": sigma, "lr": 3e-4}], lr=3e-4,
                             weight_decay=1e-4, foreach=False, fused=False)


def test_module_api_under_autocast_matches_fused_bf16_step():
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    batch = mp_like_batch(4).to(DEV)
    mod = _model(0).train()
    fus = _model(0).train()
    assert mod._engine.precision == "fp32"                  # autocast, not set_precision, picks bf16
    tr = A.FusedTrainer(fus, precision="bf16", feature_jitter_std=0.0, lr=3e-4, sigma_lr=3e-4)
    assert tr.amp_loss and tr.scaler is not None
    opt = _torch_adamw(mod)
    scaler = torch.amp.GradScaler("cuda")
    names = tr.st.names
    for it, draw in enumerate((11, 12, 13)):
        p_before = {n: p.detach().clone() for n, p in mod.named_parameters()}
        loss_m, heads_m, grads_m, norm_m = _reference_amp_step(mod, opt, scaler, batch, draw)
        assert heads_m.dtype == torch.bfloat16
        torch.manual_seed(draw)
        seed = int(torch.randint(0, 2**62, (1,)).item())   # the same draw model._run makes
        tr.forward_backward(batch, seed)
        torch.cuda.synchronize()
        assert abs(float(tr.loss) - float(loss_m)) <= 2e-6 * abs(float(loss_m)), it
        assert set(grads_m) == set(names)          # base.output_heads: unused by the hetero forward
        for n in names:
            assert torch.equal(tr.st.G.named[n], grads_m[n]), (it, n)
        tr._clip_and_update()
        torch.cuda.synchronize()
        assert float(tr.gnorm) == pytest.approx(norm_m, rel=1e-5)
        assert tr.scaler.tolist()[0] == scaler.get_scale() == 65536.0
        # the optimizers: torch's single-tensor AdamW vs the library's restatement (2 ulp of |p| on top
        # of 1e-4 of the update, as test_hip_clip_adamw_matches_torch)
        for n in names:
            pt, pf = dict(mod.named_parameters())[n].detach(), tr.st.P.named[n]
            tol = 1e-4 * (pt - p_before[n]).abs().max() + 2 * torch.finfo(torch.float32).eps * pt.abs()
            assert bool(((pt - pf).abs() <= tol).all()), (it, n, float((pt - pf).abs().max()))
        # re-synchronise the parameters so the next step's forward starts from identical weights
        with torch.no_grad():
            for n in names:
                dict(mod.named_parameters())[n].copy_(tr.st.P.named[n])


def test_module_api_under_autocast_skips_a_nonfinite_step_like_the_fused_step():
    """An infinite target makes the loss and every gradient non-finite: GradScaler skips the update and
    halves the scale in both paths."""
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    batch = mp_like_batch(4).to(DEV)
    batch.y = batch.y.clone()
    batch.y[1] = float("inf")
    mod = _model(1).train()
    fus = _model(1).train()
    tr = A.FusedTrainer(fus, precision="bf16", feature_jitter_std=0.0)
    opt = _torch_adamw(mod)
    scaler = torch.amp.GradScaler("cuda")
    p0 = {n: p.detach().clone() for n, p in mod.named_parameters()}
    f0 = tr.st.flat.clone()
    _reference_amp_step(mod, opt, scaler, batch, 5)
    torch.manual_seed(5)
    tr.step(batch, seed=int(torch.randint(0, 2**62, (1,)).item()))
    torch.cuda.synchronize()
    assert all(torch.equal(p.detach(), p0[n]) for n, p in mod.named_parameters())
    assert torch.equal(tr.st.flat, f0)
    assert scaler.get_scale() == 32768.0 and tr.scaler.tolist()[0] == 32768.0 and tr.scaler.tolist()[3] == 1.0


def test_module_api_autocast_outputs_and_embed_dtype():
    """Under autocast the heads and the embedding come back in bf16 (autocast's Linear outputs), the
    engine's own precision is untouched afterwards, and outside autocast everything is fp32."""
    from alignn_mi355x.synthetic import mp_like_batch
    batch = mp_like_batch(2).to(DEV)
    m = _model(2, dropout=0.0).eval()
    with torch.no_grad():
        m32, l32 = m(batch)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            m16, l16 = m(batch)
            e16 = m.embed(batch)
        e32 = m.embed(batch)
    assert m16.dtype == l16.dtype == e16.dtype == torch.bfloat16
    assert m32.dtype == l32.dtype == e32.dtype == torch.float32
    assert m._engine.precision == "fp32"
    assert float((m16.float() - m32).abs().max()) <= 3e-2 * float(m32.abs().max())
    with pytest.raises(NotImplementedError):
        with torch.autocast("cuda", dtype=torch.float16):
            m(batch)


def test_device_schedule_with_an_undersized_degree_bound_stays_a_permutation():
    """A host in-degree bound that is wrong (a target above the schedule's threshold): the device-built
    work list still lists every target exactly once (the over-threshold one after the zero-degree
    targets), so no attention kernel reads an unwritten entry as a node id; the error flag reports it
    at the next check (alignn_schedule_build)."""
    from alignn_mi355x import ops
    degs = torch.tensor([3, 0, 100, 7, 0, 5] * 5)
    n = degs.numel()
    dst = torch.repeat_interleave(torch.arange(n), degs)
    src = torch.randint(0, n, (dst.numel(),), generator=torch.Generator().manual_seed(1))
    g = ops.GraphCSR(torch.stack([src, dst]).to(DEV), n,
                     policy=ops.SchedulePolicy(wave_items=True, xcd_items=True, heavy_threshold=64))
    g.deg_bound = 10                       # wrong: one in-degree is 100
    assert g.device_schedule_ok()
    sc = g.schedule()
    light = g._sched[1].cpu().tolist()
    assert sc.n_light == n and sorted(light) == list(range(n))
    lit = [i for i in range(n) if 0 < int(degs[i]) <= 64]
    assert sorted(light[:len(lit)]) == lit                       # listed targets first
    assert all(int(degs[i]) in (0, 100) for i in light[len(lit):])
    with pytest.raises(RuntimeError, match="host bound"):
        g.check_indices("lg_edge_index")


@pytest.mark.parametrize("M,N,K,a_t,prec", [(768, 256, 2580, True, "fp32"), (256, 256, 23040, True, "fp32"),
                                            (2, 256, 32, True, "fp32"), (256, 36, 1920, True, "fp32"),
                                            (100, 64, 300, False, "fp32"), (768, 256, 16020, True, "bf16"),
                                            (256, 256, 184320, True, "bf16")])
def test_gemm_rowsum_is_the_bias_gradient(M, N, K, a_t, prec):
    """alignn_gemm_f32 with rowsum: the weight gradient dW = dY^T X is bitwise the plain product and
    rowsum = dY.sum(0) (the Linear's bias gradient) from the same launch, to fp32 summation order
    against an fp64 sum (split-K partials included)."""
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(M + K)
    dY = torch.randn(K, M, generator=g).to(DEV)
    X = torch.randn(K, N, generator=g).to(DEV)
    A = dY.t() if a_t else dY.t().contiguous()
    if prec == "bf16":
        dY16 = dY.bfloat16()
        A = dY16.t()
        ref_rs = dY16.double().sum(0)
    else:
        ref_rs = dY.double().sum(0)
    C0, C1 = torch.empty(M, N, device=DEV), torch.empty(M, N, device=DEV)
    rs = torch.full((M,), float("nan"), device=DEV)
    with ops.gemm_precision(prec):
        ops.gemm(A, X, C0)
        ops.gemm(A, X, C1, rowsum=rs)
    torch.cuda.synchronize()
    assert torch.equal(C0, C1)
    err = float((rs.double() - ref_rs).abs().max() / ref_rs.abs().max())
    assert err < 2e-6 * max(1.0, (K / 1000) ** 0.5), err


def test_borrowed_streams_are_the_lenders_and_the_step_is_unchanged():
    """ExecContext.borrow_streams (bench.py's secondary configurations beside the idle headline
    trainer): the borrower's side / aux streams are the lender's, a context with streams of its own
    refuses to borrow, and a step on borrowed streams gives the same bits as on its own."""
    import alignn_mi355x as A
    from alignn_mi355x import ops
    from alignn_mi355x.synthetic import mp_like_batch
    lender, own = ops.ExecContext("lender"), ops.ExecContext("own")
    own.side(DEV)
    with pytest.raises(RuntimeError):
        own.borrow_streams(lender)
    res = []
    for borrow in (False, True):
        torch.manual_seed(0)
        m = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(DEV)
        if borrow:
            m._engine.ctx.borrow_streams(lender)
        tr = A.FusedTrainer(m)
        loss = tr.forward_backward(mp_like_batch(4).to(DEV), 5).clone()
        torch.cuda.synchronize()
        if borrow:
            assert m._engine.ctx.side(DEV).cuda_stream == lender.side(DEV).cuda_stream
            assert m._engine.ctx.aux(DEV).cuda_stream == lender.aux(DEV).cuda_stream
        res.append((loss, tr.st.grad.clone()))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


def test_noisy_copies_equal_clone_then_add_noise():
    """The trainer's one-launch jitter (alignn_noisy_copy2_f32) against the two copies + two
    add_noise launches it replaced: bitwise; the sources untouched."""
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(5)
    x = torch.randn(1920, 206, generator=g).to(DEV)
    gx = torch.randn(32, 289, generator=g).to(DEV)
    x0, gx0 = x.clone(), gx.clone()
    r1, r2 = x.clone(), gx.clone()
    ops.add_noise(r1, 0.05, 123)
    ops.add_noise(r2, 0.05, 456)
    y1, y2 = ops.noisy_copies(x, 123, gx, 456, 0.05)
    torch.cuda.synchronize()
    assert torch.equal(y1, r1) and torch.equal(y2, r2)
    assert torch.equal(x, x0) and torch.equal(gx, gx0)
    z1, z2 = ops.noisy_copies(x, 123, gx, 456, 0.0)
    assert torch.equal(z1, x) and torch.equal(z2, gx)


def test_bf16_atom_edge_gradient_is_a_bf16_rounding():
    """bf16 storage (config C3): the atom blocks' edge-feature gradient stored in bf16
    (engine.bf16_atom_grad; alignn_tconv_bwd_dst_ex bit 2, alignn_gate_ln_bwd_partials_ex r_bf16 bit 1)
    against fp32 storage: the same loss (forward untouched), every gradient within bf16 rounding of
    that one tensor (normwise 1e-2), and the bf16 gradient deterministic."""
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    res = []
    for on in (False, True, True):
        torch.manual_seed(0)
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(DEV)
        model._engine.bf16_atom_grad = on
        model._engine.atom_stream = 2
        tr = A.FusedTrainer(model, precision="bf16")
        loss = tr.forward_backward(mp_like_batch(32).to(DEV), 3).clone()
        torch.cuda.synchronize()
        res.append((loss, tr.st.grad.clone()))
    (l0, g0), (l1, g1), (l2, g2) = res
    assert torch.equal(l0, l1) and torch.equal(l1, l2)
    assert torch.equal(g1, g2)
    rel = float((g1.double() - g0.double()).norm() / g0.double().norm())
    assert 0.0 < rel < 1e-2, rel


def test_batched_heads_equal_two_products():
    """engine.forward's heads: mean and logvar Linear in one batched launch over the flat parameter
    buffer (strided views) give the two separate products' bits.  (The zero-free bond gradient, gate
    dX_zero: tests/test_gpu_x_round6.py.)"""
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(9)
    B, D, Tt = 32, 256, 2
    flat = torch.randn(4096, generator=g).to(DEV)
    Wm = flat[0:Tt * D].view(Tt, D)
    bm = flat[Tt * D:Tt * D + Tt]
    off = Tt * D + Tt + 6
    Wl = flat[off:off + Tt * D].view(Tt, D)
    bl = flat[off + Tt * D:off + Tt * D + Tt]
    shared = torch.randn(B, D, generator=g).to(DEV)
    ref = torch.empty(B, 2 * Tt, device=DEV)
    ops.gemm(shared, Wm.t(), ref[:, :Tt], bias=bm)
    ops.gemm(shared, Wl.t(), ref[:, Tt:], bias=bl)
    out = torch.full((B, 2 * Tt), float("nan"), device=DEV)
    dw, db = Wl.storage_offset() - Wm.storage_offset(), bl.storage_offset() - bm.storage_offset()
    ops.gemm(shared, torch.as_strided(Wm, (2, D, Tt), (dw, 1, D)), torch.as_strided(out, (2, B, Tt), (Tt, 2 * Tt, 1)),
             bias=torch.as_strided(bm, (2, Tt), (db, 1)))
    torch.cuda.synchronize()
    assert torch.equal(out, ref)


def test_bf16_trainer_with_torch_optimizer():
    """a bf16 trainer with torch's optimizer builds and steps (no GradScaler by
    default there); asking for one with torch's optimizer is refused."""
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    torch.manual_seed(0)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 64, 1, 1, 0.0), 2).to(DEV)
    tr = A.FusedTrainer(model, precision="bf16", optimizer="torch")
    assert tr.scaler is None
    before = tr.st.flat.clone()
    loss = tr.step(mp_like_batch(4).to(DEV), seed=1)
    torch.cuda.synchronize()
    assert torch.isfinite(loss).all() and not torch.equal(before, tr.st.flat)
    with pytest.raises(ValueError):
        A.FusedTrainer(model, precision="bf16", optimizer="torch", grad_scaler=True)


@pytest.mark.parametrize("bf16", [False, True])
def test_gate_writes_the_next_blocks_active_rows(bf16):
    """alignn_gate_ln_fwd_ex2: the gate kernel's copy of the new state's active rows (Xa_out at
    outp_rows[r]) is bitwise gather_rows(Xnew, rows), and Xnew / its bf16 copy are unchanged."""
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(21)
    n, D, na = 3000, 256, 700
    rows = torch.randperm(n, generator=g)[:na].sort().values.to(torch.int32)
    cmap = torch.full((n,), -1, dtype=torch.int32)
    cmap[rows.long()] = torch.arange(na, dtype=torch.int32)
    rows, cmap = rows.to(DEV), cmap.to(DEV)
    outp = torch.randn(na, D, generator=g).to(DEV)
    R = torch.randn(n, D, generator=g).to(DEV)
    if bf16:
        R = R.to(torch.bfloat16)
    X = torch.randn(n, D, generator=g).to(DEV)
    wbeta = torch.randn(3 * D, generator=g).to(DEV) * 0.1
    lnw, lnb = torch.randn(D, generator=g).to(DEV), torch.randn(D, generator=g).to(DEV)

    def run(xa):
        Xn, st = torch.empty(n, D, device=DEV), [torch.empty(n, device=DEV) for _ in range(3)]
        X16 = torch.empty(n, D, device=DEV, dtype=torch.bfloat16) if bf16 else None
        ops.gate_ln_fwd(outp, R, wbeta, X, lnw, lnb, Xn, *st, 0.15, 77, outp_rows=cmap, Xnew16=X16, Xa_out=xa)
        return Xn, X16

    Xn0, X160 = run(None)
    xa = torch.full((na, D), float("nan"), device=DEV)
    Xn1, X161 = run(xa)
    torch.cuda.synchronize()
    assert torch.equal(Xn0, Xn1) and (not bf16 or torch.equal(X160, X161))
    assert torch.equal(xa, ops.gather_rows(Xn1, rows))
