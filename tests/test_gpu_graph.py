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
        ops.set_step_seed(tr2._seed_dev)
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
