"""Captured steps of the fused trainer (native launch plans and HIP graphs): a replayed step equals
the eager step bit for bit (same kernels, same order, same device step seed), the step seed changes
the dropout masks, and the model / optimizer state is untouched by capture."""
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _setup(seed=0, B=4):
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    torch.manual_seed(seed)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, 0.15), 2).to(DEV)
    tr = A.FusedTrainer(model)
    b = mp_like_batch(B).to(DEV)
    return model, tr, b


@pytest.mark.parametrize("B", [4, 32])
@pytest.mark.parametrize("mode", ["plan", "graph"])
def test_graph_replay_matches_eager_bitwise(mode, B):
    from alignn_mi355x import ops
    _, tr1, b1 = _setup(B=B)
    _, tr2, b2 = _setup(B=B)
    tr2.capture(b2, mode=mode)
    assert torch.equal(tr1.st.flat, tr2.st.flat)          # capture leaves the weights as they were
    for i, s in enumerate((11, 12, 13)):
        # eager reference with the same device step seed the replay uses
        tr1.use_step_seed(tr2._seed_dev)
        tr2._seed_dev.fill_(s)
        l1 = tr1.forward_backward(b1, 0).clone()
        tr1._clip_and_update()
        l2 = tr2.step(b2, seed=s).clone()
        torch.cuda.synchronize()
        assert torch.equal(l1, l2), i
        assert torch.equal(tr1.st.grad, tr2.st.grad), i
        assert torch.equal(tr1.st.flat, tr2.st.flat), i
    ops.set_step_seed(None)


@pytest.mark.parametrize("mode", ["plan", "graph"])
def test_graph_step_seed_changes_masks(mode):
    from alignn_mi355x import ops
    _, tr, b = _setup()
    tr.capture(b, mode=mode)
    flat0 = tr.st.flat.clone()
    tr.step(b, seed=1)
    g1 = tr.st.grad.clone()
    tr.st.flat.copy_(flat0)
    tr.step(b, seed=2)
    g2 = tr.st.grad.clone()
    torch.cuda.synchronize()
    assert not torch.equal(g1, g2)
    ops.set_step_seed(None)


def test_side_stream_overlap_is_bitwise_neutral():
    """Weight-gradient work on the side stream gives the same bits as all on one stream."""
    _, tr1, b1 = _setup()
    _, tr2, b2 = _setup()
    tr2.model._engine.overlap = False
    l1 = tr1.forward_backward(b1, 7)
    l2 = tr2.forward_backward(b2, 7)
    torch.cuda.synchronize()
    assert torch.equal(l1, l2)
    assert torch.equal(tr1.st.grad, tr2.st.grad)


def test_plan_structure():
    """The recorded forward/backward plan holds the whole step on three streams (critical path, the
    weight-gradient side stream, the aux stream of the deferred angle-encoder backward) with its
    fork/join edges; the update plan is one stream."""
    from alignn_mi355x import ops
    from alignn_mi355x.trainer import plan_info
    _, tr, b = _setup()
    tr.capture(b, mode="plan")
    fb, up = (plan_info(p) for p in tr._graph[3])
    assert fb["launches"] > 150 and fb["streams"] == 3 and fb["edges"] >= 8, fb
    assert up["launches"] >= 3 and up["streams"] == 1 and up["edges"] == 0, up
    tr.release_capture()
    assert tr._graph is None
    ops.set_step_seed(None)


def test_plan_needs_library_optimizer():
    import alignn_mi355x as A
    from alignn_mi355x.synthetic import mp_like_batch
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 64, 1, 4, 0.0), 2).to(DEV)
    tr = A.FusedTrainer(model, optimizer="torch")
    with pytest.raises(ValueError):
        tr.capture(mp_like_batch(2).to(DEV), mode="plan")


def test_two_captured_trainers_interleave_bitwise():
    """Two trainers (B = 4 and the bench's B = 32) hold captured plans at the same time; their
    replays interleave, each matches an eager twin bit for bit (no shared workspace, stream or seed)."""
    trs = []
    for B in (4, 32):
        _, te, be = _setup(B=B)
        _, tp, bp = _setup(B=B)
        tp.capture(bp)
        te.use_step_seed(tp._seed_dev)
        trs.append((te, be, tp, bp))
    for s in (21, 22):
        for te, be, tp, bp in trs:
            tp._seed_dev.fill_(s)
            le = te.forward_backward(be, 0).clone()
            te._clip_and_update()
            lp = tp.step(bp, seed=s).clone()
            torch.cuda.synchronize()
            assert torch.equal(le, lp)
            assert torch.equal(te.st.flat, tp.st.flat)
    for _, _, tp, _ in trs:
        tp.release_capture()


def test_plan_ownership_check():
    """alignn_plan_check_ptrs: a recorded launch into a buffer outside the declared ranges is
    reported with its address; declared, it passes."""
    import ctypes
    from alignn_mi355x import _lib, ops
    from alignn_mi355x.trainer import _record_plan
    lib = _lib.lib()
    a = torch.empty(1000, device=DEV)
    b = torch.empty(1000, device=DEV)
    ctx = ops.ExecContext("t")
    with ops.using(ctx), ops.recording():
        plan = _record_plan(lambda: (ops.zero_(a), ops.copy_(b, a)))
    try:
        def check(tensors):
            rs = [v for t in tensors for v in (t.data_ptr(), t.data_ptr() + 4 * t.numel())]
            arr = (ctypes.c_uint64 * len(rs))(*rs)
            bad, idx, n = ctypes.c_uint64(), ctypes.c_int64(), ctypes.c_int64()
            rc = lib.alignn_plan_check_ptrs(plan, arr, len(tensors), ctypes.byref(bad), ctypes.byref(idx),
                                            ctypes.byref(n))
            return rc, bad.value, idx.value, n.value
        assert check([a, b])[0] == 0 and check([a, b])[3] == 3
        rc, bad, idx, _ = check([a])
        assert rc != 0 and bad == b.data_ptr() and idx == 1
    finally:
        lib.alignn_plan_destroy(plan)
    torch.cuda.synchronize()


def _twin_step(te, tp, b, s):
    """Eager step of ``te`` on ``b`` with the device step seed ``tp``'s replay uses."""
    te.use_step_seed(tp._seed_dev)
    tp._seed_dev.fill_(s)
    le = te.forward_backward(b, 0).clone()
    te._clip_and_update()
    return le


def test_rebind_new_batches_replay_bitwise():
    """A captured plan re-bound to fresh batches of the same signature (FusedTrainer._rebind: copied
    into the captured batch) equals the eager step on each of them bit for bit — including batches
    collated on the device from an HBM store and prepared on a loader stream (engine.prepare_batch),
    as the reference's loop over fresh batches (train.py:639-711) runs at plan speed."""
    import numpy as np
    from alignn_mi355x import ops
    from alignn_mi355x.data import Data
    from alignn_mi355x.engine import prepare_batch
    from alignn_mi355x.store import GraphStore
    from alignn_mi355x.synthetic import mp_like_batch, mp_like_graph
    _, te, _ = _setup(B=8)
    _, tp, bp = _setup(B=8)
    tp.capture(bp)
    # re-binding copies only into the buffers the plans touch: the raw line-graph index and angle
    # features are read when the cache is built (CSR, target-sorted angle rows), never by the step.
    # The plans read the trainer's private copy of the captured batch (the slot), never bp itself
    used, slot = tp._graph[5], tp._graph[2]
    assert slot is not bp and slot.x.data_ptr() != bp.x.data_ptr()
    assert slot.x.data_ptr() in used and slot.y.data_ptr() in used
    assert slot.lg_edge_index.data_ptr() not in used and slot.lg_edge_attr.data_ptr() not in used
    assert bp.x.data_ptr() not in used
    keys = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y")
    store = GraphStore.from_data_list([Data(**{k: getattr(mp_like_graph(100 + g), k) for k in keys})
                                       for g in range(24)], DEV)
    loader = torch.cuda.Stream()
    rng = np.random.default_rng(5)
    batches = [mp_like_batch(8, first=40).to(DEV)]
    for _ in range(3):
        with torch.cuda.stream(loader):
            b = store.collate(rng.choice(24, size=8, replace=False))
        prepare_batch(b, loader)
        batches.append(b)
    for i, b in enumerate(batches):
        s = 31 + i
        lp = tp.step(b, seed=s).clone()
        le = _twin_step(te, tp, b, s)
        torch.cuda.synchronize()
        assert torch.equal(le, lp), i
        assert torch.equal(te.st.grad, tp.st.grad), i
        assert torch.equal(te.st.flat, tp.st.flat), i
    assert tp.rebinds == len(batches) and tp.rebind_misses == 0
    # a batch of another signature runs eagerly (nothing copied) and is still the eager step
    b3 = mp_like_batch(3, first=7).to(DEV)
    tp._seed_dev.fill_(0)   # the eager path mixes the host seed with the device one, as the twin does
    lp = tp.step(b3, seed=50).clone()
    te.use_step_seed(tp._seed_dev)
    le = te.forward_backward(b3, 50).clone()
    te._clip_and_update()
    torch.cuda.synchronize()
    assert tp.rebind_misses == 1
    assert torch.equal(le, lp) and torch.equal(te.st.flat, tp.st.flat)
    tp.release_capture()
    ops.set_step_seed(None)


def test_set_lr_reaches_a_captured_plan():
    """Learning rates are a device pair read by the AdamW kernel: set_lr after capture changes the
    replayed update exactly as it changes the eager one (no re-capture; train.py:1641-1652)."""
    from alignn_mi355x import ops
    _, te, b1 = _setup()
    _, tp, b2 = _setup()
    tp.capture(b2)
    for i, lr in enumerate((3e-4, 1e-3, 5e-5)):
        te.set_lr(lr, lr / 3)
        tp.set_lr(lr, lr / 3)
        lp = tp.step(b2, seed=60 + i).clone()
        le = _twin_step(te, tp, b1, 60 + i)
        torch.cuda.synchronize()
        assert torch.equal(le, lp) and torch.equal(te.st.flat, tp.st.flat), i
    # and it matters: a different rate gives different parameters
    flat = tp.st.flat.clone()
    tp.set_lr(1e-2)
    tp.step(b2, seed=70)
    te.set_lr(1e-3)
    _twin_step(te, tp, b1, 70)
    torch.cuda.synchronize()
    assert not torch.equal(te.st.flat, tp.st.flat) and not torch.equal(flat, tp.st.flat)
    tp.release_capture()
    ops.set_step_seed(None)


def test_larger_miss_then_rebind_hit_bitwise():
    """A re-bind miss on a LARGER batch runs eagerly in the captured trainer's context; its bigger
    workspaces must not replace the ones the plan holds (ExecContext.freeze), so the next replay and
    re-bound hit still equal the eager twin bit for bit."""
    from alignn_mi355x import ops
    from alignn_mi355x.synthetic import mp_like_batch
    _, te, _ = _setup(B=8)
    _, tp, bp = _setup(B=8)
    tp.capture(bp)
    big = mp_like_batch(20, first=300).to(DEV)
    hit = mp_like_batch(8, first=500).to(DEV)
    for i, b in enumerate((big, hit, bp, big, hit)):
        s = 80 + i
        if b is big:
            tp._seed_dev.fill_(0)
            lp = tp.step(b, seed=s).clone()
            te.use_step_seed(tp._seed_dev)
            le = te.forward_backward(b, s).clone()
            te._clip_and_update()
        else:
            lp = tp.step(b, seed=s).clone()
            le = _twin_step(te, tp, b, s)
        torch.cuda.synchronize()
        assert torch.equal(le, lp), i
        assert torch.equal(te.st.grad, tp.st.grad), i
        assert torch.equal(te.st.flat, tp.st.flat), i
    assert tp.rebind_misses == 2 and tp.rebinds >= 2
    tp.release_capture()
    ops.set_step_seed(None)


@pytest.mark.parametrize("path", ["sample_weights", "no_capture"])
def test_loader_prepared_batch_on_eager_paths(path):
    """A batch collated and prepared on a loader stream is waited for and kept alive on every path
    that reads it (engine.adopt): the KNN-weighted eager step of a captured trainer and a trainer with
    no capture equal the same step on the same batch prepared on the main stream."""
    import numpy as np
    from alignn_mi355x import ops
    from alignn_mi355x.data import Data
    from alignn_mi355x.engine import prepare_batch
    from alignn_mi355x.store import GraphStore
    from alignn_mi355x.synthetic import mp_like_batch, mp_like_graph
    keys = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y")
    store = GraphStore.from_data_list([Data(**{k: getattr(mp_like_graph(200 + g), k) for k in keys})
                                       for g in range(16)], DEV)
    idx = np.random.default_rng(3).choice(16, size=8, replace=False)
    loader = torch.cuda.Stream()
    _, t1, _ = _setup(B=8)
    _, t2, b2 = _setup(B=8)
    if path == "sample_weights":
        t2.capture(b2)
    w = torch.linspace(0.5, 1.5, 8, device=DEV) if path == "sample_weights" else None
    for i in range(2):
        with torch.cuda.stream(loader):
            bl = store.collate(idx)
            torch.cuda._sleep(2_000_000)    # the loader is still busy when the step is queued
        prepare_batch(bl, loader)
        bm = store.collate(idx)
        prepare_batch(bm)
        t1.use_step_seed(None)
        t2.use_step_seed(None)
        ops.set_step_seed(None)
        l1 = t1.step(bm, seed=90 + i, sample_weights=w).clone()
        l2 = t2.step(bl, seed=90 + i, sample_weights=w).clone()
        del bl
        torch.cuda.synchronize()
        assert torch.equal(l1, l2), i
        assert torch.equal(t1.st.flat, t2.st.flat), i
    t2.release_capture()


def test_bucketed_dp_plan_replay_bitwise():
    """The data-parallel step with the bucketed gradient exchange (dp.GradBuckets: three captured
    phases, the first bucket's all_reduce issued between the per-layer backward and the tail) equals
    the plain eager step bit for bit (one rank: the reductions are identities)."""
    import socket
    import torch.distributed as dist
    from alignn_mi355x import dp, ops
    from alignn_mi355x.layout import bucket_split
    with socket.socket() as sk:
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        _, te, b1 = _setup(B=8)
        _, tp, b2 = _setup(B=8)
        tp.grad_buckets = dp.GradBuckets(tp.st.grad, bucket_split(tp.model.config, True), 1)
        tp.capture(b2)
        assert len(tp._graph[3]) == 3
        for i, s in enumerate((41, 42, 43)):
            lp = tp.step(b2, seed=s).clone()
            le = _twin_step(te, tp, b1, s)
            torch.cuda.synchronize()
            assert torch.equal(le, lp), i
            assert torch.equal(te.st.grad, tp.st.grad), i
            assert torch.equal(te.st.flat, tp.st.flat), i
        tp.release_capture()
        # the eager bucketed step too
        tp.use_step_seed(None)
        te.use_step_seed(None)
        ops.set_step_seed(None)
        lp = tp.step(b2, seed=50).clone()
        le = te.step(b1, seed=50).clone()
        torch.cuda.synchronize()
        assert torch.equal(le, lp) and torch.equal(te.st.flat, tp.st.flat)
    finally:
        dist.destroy_process_group()
        ops.set_step_seed(None)
