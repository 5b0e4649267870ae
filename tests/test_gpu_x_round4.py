"""Round-4 GPU checks: GradScaler semantics of the bf16 step (train.py:690-695), the captured plan's
stream-dependency validator, KNN-weighted steps on the replayed plan (train.py:660-674), the filtered
re-binding copy against copying every buffer, and a C3-size (B = 256) fp32 forward against the
reference's CPU path (the oracle in fp32)."""
import pytest
import torch

from _golden_util import rel_err

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _trainer(B=4, precision=None, seed=0, first=0, **kw):
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    torch.manual_seed(seed)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(DEV)
    tr = A.FusedTrainer(model, precision=precision, **kw)
    return tr, mp_like_batch(B, first=first).to(DEV)


# ------------------------------------------------------------------------------------------------
# GradScaler (torch.amp defaults: init 2^16, growth 2 every 2000 clean steps, backoff 0.5)
# ------------------------------------------------------------------------------------------------
def test_grad_scaler_skips_a_nonfinite_step_eager():
    """One gradient set to inf: scaler.step skips AdamW (parameters, moments and the step count stay),
    update halves the scale; the next clean step updates.  A clean step equals the scaler-free step."""
    tr, b = _trainer(precision="bf16")
    assert tr.scaler is not None                                   # bf16 = the reference's autocast path
    ref, _ = _trainer(precision="bf16", grad_scaler=False)
    tr.forward_backward(b, 5)
    ref.forward_backward(b, 5)
    tr._clip_and_update()
    ref._clip_and_update()
    torch.cuda.synchronize()
    assert torch.equal(tr.st.flat, ref.st.flat) and torch.equal(tr.exp_avg_sq, ref.exp_avg_sq)
    assert tr.scaler.tolist() == [65536.0, 1.0, 0.0, 0.0]
    p0, m0, v0, s0 = tr.st.flat.clone(), tr.exp_avg.clone(), tr.exp_avg_sq.clone(), tr.hip_step.clone()
    tr.forward_backward(b, 6)
    tr.st.grad[12345] = float("inf")
    tr._clip_and_update()
    torch.cuda.synchronize()
    assert torch.equal(tr.st.flat, p0) and torch.equal(tr.exp_avg, m0) and torch.equal(tr.exp_avg_sq, v0)
    assert torch.equal(tr.hip_step, s0)
    assert tr.scaler.tolist() == [32768.0, 0.0, 1.0, 1.0]
    tr.forward_backward(b, 7)
    tr._clip_and_update()
    torch.cuda.synchronize()
    assert not torch.equal(tr.st.flat, p0) and float(tr.hip_step) == float(s0) + 1
    assert tr.scaler.tolist() == [32768.0, 1.0, 0.0, 1.0]


def test_grad_scaler_overflow_of_the_scaled_gradient_counts():
    """unscale_ flags a gradient whose SCALED value is not finite: 1e36 * 65536 overflows fp32."""
    tr, b = _trainer(precision="bf16")
    tr.forward_backward(b, 5)
    p0 = tr.st.flat.clone()
    tr.st.grad[7] = 1e36
    tr._clip_and_update()
    torch.cuda.synchronize()
    assert torch.equal(tr.st.flat, p0) and tr.scaler.tolist()[2:] == [1.0, 1.0]


def test_grad_scaler_growth_interval():
    tr, b = _trainer(precision="bf16", growth_interval=2)
    for s in range(3):
        tr.forward_backward(b, s)
        tr._clip_and_update()
    torch.cuda.synchronize()
    assert tr.scaler.tolist() == [131072.0, 1.0, 0.0, 0.0]


def test_grad_scaler_on_the_replayed_plan():
    """A NaN input feature makes every gradient NaN; the replayed step is skipped on the device (no
    host sync), then the restored batch trains again."""
    tr, b = _trainer(precision="bf16")
    tr.capture(b)
    tr.step(b, seed=1)
    torch.cuda.synchronize()
    p0, m0, s0 = tr.st.flat.clone(), tr.exp_avg.clone(), float(tr.hip_step)
    x0 = b.x[0, 0].item()
    b.x[0, 0] = float("nan")
    tr.step(b, seed=2)
    torch.cuda.synchronize()
    assert torch.equal(tr.st.flat, p0) and torch.equal(tr.exp_avg, m0) and float(tr.hip_step) == s0
    assert tr.scaler.tolist()[0] == 32768.0 and tr.scaler.tolist()[3] == 1.0
    b.x[0, 0] = x0
    tr.step(b, seed=3)
    torch.cuda.synchronize()
    assert not torch.equal(tr.st.flat, p0) and float(tr.hip_step) == s0 + 1
    assert torch.isfinite(tr.st.flat).all()


# ------------------------------------------------------------------------------------------------
# Plan dependency validator (alignn_plan_check_deps)
# ------------------------------------------------------------------------------------------------
def _capture_two_streams(fork_noted: bool, join_noted: bool, tail_kernel: bool):
    from alignn_mi355x import _lib, ops
    from alignn_mi355x import trainer as T
    ctx = ops.ExecContext("deps-test")
    side = ctx.side(torch.device(DEV))
    x = torch.ones(1 << 16, device=DEV)
    y = torch.ones(1 << 16, device=DEV)
    z = torch.ones(1 << 16, device=DEV)
    g = torch.cuda.CUDAGraph(keep_graph=True)
    torch.cuda.synchronize()

    def fn():
        cur = torch.cuda.current_stream()
        ops.zero_(x)
        if fork_noted:
            ops.stream_wait(side, cur)
        else:
            side.wait_stream(cur)                   # a torch-level wait the plan never hears of
        with torch.cuda.stream(side):
            ops.add_(y, x)
        if join_noted:
            ops.stream_wait(cur, side)
        else:
            cur.wait_stream(side)
        if tail_kernel:
            ops.add_(z, y)

    with ops.using(ctx), ops.recording():
        with torch.cuda.graph(g):
            plan = T._record_plan(fn)
    torch.cuda.synchronize()
    return g, plan, _lib, T


@pytest.mark.parametrize("fork_noted,join_noted,tail,ok", [
    (True, True, True, True), (True, True, False, True),
    (False, True, True, False),    # the graph orders x's kernel before the side kernel, the plan does not
    (True, False, True, False),    # side kernel -> tail kernel edge missing
    (True, False, False, False)])  # nothing after the join: the plan ends with the side slot unjoined
def test_plan_dependency_validator(fork_noted, join_noted, tail, ok):
    g, plan, _lib, T = _capture_two_streams(fork_noted, join_noted, tail)
    try:
        if ok:
            assert T._check_deps(g, plan, "test") >= 1
        else:
            with pytest.raises(RuntimeError, match="misses a stream dependency"):
                T._check_deps(g, plan, "test")
    finally:
        _lib.lib().alignn_plan_destroy(plan)


def test_every_trainer_capture_passes_the_validator():
    """The real captures (plain, bucketed data-parallel phases at world 1) pass: capture() runs the
    validator on every phase and would raise."""
    from alignn_mi355x.dp import GradBuckets
    from alignn_mi355x.layout import bucket_split
    tr, b = _trainer(B=4)
    tr.capture(b)
    tr.step(b, seed=1)
    tr2, b2 = _trainer(B=4)
    tr2.grad_buckets = GradBuckets(tr2.st.grad, bucket_split(tr2.model.config, True), 1)
    tr2.capture(b2)
    assert len(tr2._graph[3]) == 3
    tr3, b3 = _trainer(B=32, precision="bf16")
    tr3.capture(b3)
    torch.cuda.synchronize()


# ------------------------------------------------------------------------------------------------
# KNN-weighted steps on the plan path; filtered vs full re-binding copy
# ------------------------------------------------------------------------------------------------
def test_weighted_replay_matches_eager_weighted_step():
    from alignn_mi355x import ops
    from alignn_mi355x.synthetic import mp_like_batch
    tr1, b1 = _trainer(B=8)
    tr2, b2 = _trainer(B=8)
    tr2.capture(b2, weighted=True)
    b3 = mp_like_batch(8, first=500).to(DEV)          # same signature, other graphs: re-bound
    gen = torch.Generator().manual_seed(3)
    for i, (s, bb1, bb2) in enumerate(((21, b1, b2), (22, b1, b2), (23, b3, b3))):
        w = (0.5 + torch.rand(8, generator=gen)).to(DEV)
        tr1.use_step_seed(tr2._seed_dev)
        tr2._seed_dev.fill_(s)
        l1 = tr1.forward_backward(bb1, 0, sample_weights=w).clone()
        tr1._clip_and_update()
        n0 = tr2.replays
        l2 = tr2.step(bb2, seed=s, sample_weights=w).clone()
        torch.cuda.synchronize()
        assert tr2.replays == n0 + 1, i                # replayed, not an eager fallback
        assert torch.equal(l1, l2), i
        assert torch.equal(tr1.st.grad, tr2.st.grad), i
        assert torch.equal(tr1.st.flat, tr2.st.flat), i
    assert tr2.rebinds >= 1
    n0 = tr2.replays
    tr2.step(b2, seed=30)                               # unweighted step on a weighted capture: eager
    assert tr2.replays == n0
    ops.set_step_seed(None)


def test_filtered_rebind_copy_equals_copying_every_buffer():
    """alignn_plan_refs restricts the re-binding copy to the buffers some recorded launch points into;
    the same replay with every batch and cache buffer copied gives the same bits."""
    from alignn_mi355x.synthetic import mp_like_batch
    tr1, b1 = _trainer(B=8)
    tr2, b2 = _trainer(B=8)
    tr1.capture(b1)
    tr2.capture(b2)
    tr2.rebind_copy_all = True
    for s, first in ((41, 700), (42, 900)):
        nb = mp_like_batch(8, first=first).to(DEV)
        tr1.step(nb, seed=s)
        tr2.step(nb, seed=s)
    torch.cuda.synchronize()
    assert tr1.rebinds == tr2.rebinds == 2
    assert torch.equal(tr1.st.grad, tr2.st.grad) and torch.equal(tr1.st.flat, tr2.st.flat)


# ------------------------------------------------------------------------------------------------
# C3-size wiring against the reference's CPU path
# ------------------------------------------------------------------------------------------------
@pytest.mark.timeout(400)
def test_c3_size_fp32_forward_vs_oracle():
    """B = 256 MP-like graphs under the PyG offset rule (16,020 active bonds, 2,027,520 triplets),
    D256/H4/L4, fp32, dropout 0: the engine's (mean, logvar) against the oracle's fp32 forward on the
    host (the reference's CPU path), tolerance 1e-4 relative (north_star).  Pins the compacted C3
    line-graph wiring to something other than the engine itself."""
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    from oracle import model_ref
    from oracle.pyg_ref import RefData
    torch.manual_seed(256)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.0), 2)
    st = {k: v.detach().clone() for k, v in model.state_dict().items()}
    cpu_batch = mp_like_batch(256, lg_offset="num_nodes")
    assert cpu_batch.lg_edge_index.size(1) == 2027520
    model.to(DEV).eval()
    with torch.no_grad():   # (Batch.to moves in place: a separate copy for the device)
        mean, logvar = model(mp_like_batch(256, lg_offset="num_nodes").to(DEV))
    torch.cuda.synchronize()
    mean, logvar = mean.cpu(), logvar.cpu()
    rb = RefData(**{k: getattr(cpu_batch, k) for k in cpu_batch.keys()})
    rb.num_graphs = 256
    with torch.no_grad():
        rmean, rlogvar = model_ref.hetero_forward(st, rb, 4)
    assert rel_err(mean, rmean) < 1e-4
    assert rel_err(logvar, rlogvar) < 1e-4


# ------------------------------------------------------------------------------------------------
# Store batches prepared without device->host copies (device-built schedules, host-sized compaction)
# ------------------------------------------------------------------------------------------------
def _host_and_device_lists(g):
    import numpy as np
    from alignn_mi355x import ops
    off = g.off_dst.cpu().numpy().astype(np.int64)
    deg = off[1:] - off[:-1]
    po = g.policy
    light, heavy = ops.schedule_lists(deg, po.heavy_threshold, po.wave_items, po.xcd_items and po.wave_items,
                                      po.xcds, g.xcd_chunk)
    g._sched = None
    g.deg_bound = int(deg.max()) if len(deg) else 0
    sc = g.schedule()
    dev = g._sched[1].cpu().numpy().astype(np.int64)
    assert sc.n_heavy == 0 and len(heavy) == 0 and sc.n_light == g.n
    return deg, off, light, dev


@pytest.mark.parametrize("which,B,lg_offset,chunk", [("lg", 32, "num_nodes", 1), ("ag", 32, "num_nodes", 4),
                                                     ("lg", 4, "num_edges", 1), ("lg", 1, "num_nodes", 1),
                                                     ("ag", 256, "num_nodes", 4), ("lg", 256, "num_nodes", 1)])
def test_device_schedule_equals_host_lists(which, B, lg_offset, chunk):
    """alignn_schedule_build against ops.schedule_lists: the same list, element for element (a stable
    order: ties in ascending id), and so at every position a target of the same in-degree from the
    same XCD id range."""
    import numpy as np
    from alignn_mi355x.engine import batch_cache
    from alignn_mi355x.synthetic import mp_like_batch
    b = mp_like_batch(B, lg_offset=lg_offset).to(DEV)
    bc = batch_cache(b)
    g = bc.lg if which == "lg" else bc.ag
    g.xcd_chunk = chunk
    deg, off, host, dev = _host_and_device_lists(g)
    assert sorted(dev.tolist()) == list(range(g.n))
    assert np.array_equal(dev, host)
    assert np.array_equal(deg[dev], deg[host])
    tot = int(off[-1])
    bounds = np.asarray([0] + [int(np.searchsorted(off[1:], tot * x // 8, side="right")) for x in range(1, 8)]
                        + [g.n])
    rng_of = lambda ids: np.searchsorted(bounds, ids, side="right") - 1   # noqa: E731
    lit = deg[host] > 0
    if int(lit.sum()) > 8:
        assert np.array_equal(rng_of(dev[lit]), rng_of(host[lit]))


def test_store_batch_prepares_without_a_host_sync_and_trains_bitwise_equal():
    """A store-collated batch carries host bounds (in-degrees, compacted line-graph size): collate +
    prepare_batch then run under torch's sync debug mode set to error (no .item / .cpu / nonzero), and
    the training step on it equals the step on the same batch prepared the synchronous way."""
    import numpy as np
    import alignn_mi355x as A
    from alignn_mi355x.engine import prepare_batch
    from alignn_mi355x.store import GraphStore
    from alignn_mi355x.synthetic import mp_like_graph
    st = GraphStore.from_data_list([mp_like_graph(g) for g in range(40)], DEV)
    sel = np.random.default_rng(3).choice(40, size=32, replace=False)
    st.collate(sel)                      # first use: the store's one-time per-graph statistics
    torch.cuda.synchronize()
    torch.cuda.set_sync_debug_mode("error")
    try:
        b_fast = st.collate(sel)
        prepare_batch(b_fast)
    finally:
        torch.cuda.set_sync_debug_mode("default")
    assert b_fast._alignn_cache.lg.device_schedule_ok() and b_fast._alignn_cache.ag.device_schedule_ok()
    b_slow = st.collate(sel)
    del b_slow._alignn_hints
    prepare_batch(b_slow)
    assert b_slow._alignn_cache.lg.n == b_fast._alignn_cache.lg.n == 2580
    grads = []
    for b in (b_fast, b_slow):
        torch.manual_seed(0)
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(DEV)
        tr = A.FusedTrainer(model)
        tr.forward_backward(b, 5)
        grads.append(tr.st.grad.clone())
    torch.cuda.synchronize()
    assert torch.equal(grads[0], grads[1])


def test_batch_prepared_on_a_dedicated_queue_stream_equals_the_current_stream():
    """ops.dedicated_stream (alignn_stream_create_dedicated: a CU-masked stream on a hardware queue of
    its own, bench's loader): one per device, reused; a store batch collated and prepared on it has the
    same line-graph CSR and work list as one prepared on the current stream."""
    import numpy as np
    from alignn_mi355x import ops
    from alignn_mi355x.engine import prepare_batch
    from alignn_mi355x.store import GraphStore
    from alignn_mi355x.synthetic import mp_like_graph
    s1 = ops.dedicated_stream(DEV)
    assert ops.dedicated_stream(DEV).cuda_stream == s1.cuda_stream
    assert s1.cuda_stream != torch.cuda.current_stream().cuda_stream
    st = GraphStore.from_data_list([mp_like_graph(g) for g in range(24)], DEV)
    sel = np.random.default_rng(5).choice(24, size=16, replace=False)
    ref = st.collate(sel)
    prepare_batch(ref)
    with torch.cuda.stream(s1):
        b = st.collate(sel)
    prepare_batch(b, s1)
    torch.cuda.current_stream().wait_stream(s1)
    torch.cuda.synchronize()
    for name in ("lg", "ag"):
        g, r = getattr(b._alignn_cache, name), getattr(ref._alignn_cache, name)
        assert g.n == r.n and g.m == r.m
        for f in ("off_dst", "src_at", "off_src", "pos_src"):
            assert torch.equal(getattr(g, f), getattr(r, f)), (name, f)


# ------------------------------------------------------------------------------------------------
# bf16 edge-feature rows in the atom-graph attention (alignn_tconv_fwd_ex / _bwd_dst_ex)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("drop", [0.0, 0.15])
def test_atom_attention_bf16_feature_rows_bitwise_vs_fp32_on_rounded_rows(drop):
    """The bond-state rows read as bf16 (config C3: autocast casts the bond state for edge_proj) give
    bit for bit what the fp32 kernels give on the same rows widened to fp32 (bf16 -> fp32 is exact,
    the arithmetic is unchanged): forward outputs, and the target-side backward including the
    edge-feature gradient written through feat_row."""
    from alignn_mi355x import ops
    from alignn_mi355x.engine import prepare_batch
    from alignn_mi355x.synthetic import mp_like_batch
    ops.set_step_seed(None)
    b = mp_like_batch(8).to(DEV)
    g = prepare_batch(b).ag
    n, m, D, H = g.n, g.m, 256, 4
    gen = torch.Generator(device="cpu").manual_seed(21)
    r = lambda *s: torch.randn(*s, generator=gen).to(DEV)   # noqa: E731
    QKVR, U, wbar, Vd = r(n, 4 * D), r(n, H, D) * 0.1, r(D) * 0.1, r(n, H, D) * 0.1
    F16 = r(m, D).bfloat16()
    dout, outs = r(n, D), []
    for F in (F16, F16.float()):
        aggV, S = torch.empty(n, D, device=DEV), torch.empty(n, H, D, device=DEV)
        sumA, mstat, den = (torch.empty(n, H, device=DEV) for _ in range(3))
        ops.tconv_fwd(g, D, H, QKVR, U, wbar, F, g.perm_dst, aggV, S, sumA, mstat, den, drop, 99)
        dq = torch.empty(n, D, device=DEV)
        Sz = torch.empty(n, H, D, device=DEV)
        sigz = torch.empty(n, H, device=DEV)
        dz_e, al_e = torch.empty(m, H, device=DEV), torch.empty(m, H, device=DEV)
        dF = torch.zeros(m, D, device=DEV)
        ops.tconv_bwd_dst(g, D, H, QKVR, U, Vd, wbar, F, g.perm_dst, dout, aggV, mstat, den, dq, Sz, sigz, dz_e,
                          al_e, dF, 1, drop, 99)
        outs.append((aggV, S, sumA, mstat, den, dq, Sz, sigz, dz_e, al_e, dF))
    torch.cuda.synchronize()
    for i, (x, y) in enumerate(zip(*outs)):
        assert torch.equal(x, y), i


def test_source_side_backward_bf16_rows_bitwise_vs_fp32_on_rounded_rows():
    """alignn_tconv_bwd_src_by_bf16 (the line graph's source-side backward at bf16 storage: Q and dout
    gathered from bf16 copies) equals the fp32 kernel on the same rows widened to fp32, bit for bit."""
    from alignn_mi355x import ops
    from alignn_mi355x.engine import prepare_batch
    from alignn_mi355x.synthetic import mp_like_batch
    b = mp_like_batch(8).to(DEV)
    g = prepare_batch(b).lg
    n, m, D, H = g.n, g.m, 256, 4
    gen = torch.Generator(device="cpu").manual_seed(31)
    QKV16 = torch.randn(n, 3 * D, generator=gen).to(DEV).bfloat16()
    dout16 = torch.randn(n, D, generator=gen).to(DEV).bfloat16()
    dz, al = torch.randn(m, H, generator=gen).to(DEV), torch.rand(m, H, generator=gen).to(DEV)
    out = []
    for bf in (True, False):
        dKV = torch.empty(n, 2 * D, device=DEV)
        if bf:
            ops.tconv_bwd_src(g, D, H, QKV16.float(), dout16.float(), dz, al, dKV, Q16=QKV16[:, :D], dout16=dout16)
        else:
            ops.tconv_bwd_src(g, D, H, QKV16.float(), dout16.float(), dz, al, dKV)
        out.append(dKV)
    torch.cuda.synchronize()
    assert torch.equal(out[0], out[1])
