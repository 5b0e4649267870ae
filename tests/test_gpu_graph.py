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
    """The recorded forward/backward plan holds the whole step on two streams (critical path +
    weight-gradient side stream) with its fork/join edges; the update plan is one stream."""
    from alignn_mi355x import ops
    from alignn_mi355x.trainer import plan_info
    _, tr, b = _setup()
    tr.capture(b, mode="plan")
    fb, up = (plan_info(p) for p in tr._graph[3])
    assert fb["launches"] > 150 and fb["streams"] == 2 and fb["edges"] >= 8, fb
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
