"""Recorded inference forwards (alignn_mi355x/infer.py): the forward-only consumers of the hot path —
``eval_epoch_hetero`` (train.py:726-846), ``ensemble_collect`` (:849-904), ``compute_global_knn_weights``
(:930-1010), ``predict.ensemble_predict`` (predict.py:582) — replay a native launch plan of the forward
once a batch signature repeats.  Every replay is bitwise the eager forward: the captured batch itself,
a re-bound batch of the same signature, the module API in fp32 and under bf16 autocast, embed mode,
and the concurrent ensemble members."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _model(dims=(206, 36, 11, 289, 2, 256, 2, 4, 0.15), seed=0):
    import alignn_mi355x as A
    torch.manual_seed(seed)
    return A.HeteroAlignnRegressor(A.AlignnRegressor(*dims), 2).to(DEV).eval()


def _eager(model, batch, mode="hetero", amp=False):
    from alignn_mi355x import infer
    prev = infer.ENABLED
    infer.ENABLED = False
    try:
        with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            r = model.embed(batch) if mode == "embed" else torch.cat(model(batch), 1)
        torch.cuda.synchronize()
        return r.clone()
    finally:
        infer.ENABLED = prev


def _planned(model, batch, mode="hetero", amp=False):
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
        r = model.embed(batch) if mode == "embed" else torch.cat(model(batch), 1)
    torch.cuda.synchronize()
    return r


@pytest.mark.parametrize("mode,amp", [("hetero", False), ("embed", False), ("hetero", True)])
def test_module_eval_forward_replays_bitwise(mode, amp):
    from alignn_mi355x.synthetic import mp_like_batch
    model = _model()
    b1 = mp_like_batch(8).to(DEV)
    b2 = mp_like_batch(8, first=100).to(DEV)   # the same signature, other features
    ref1, ref2 = _eager(model, b1, mode, amp), _eager(model, b2, mode, amp)
    outs = [_planned(model, b, mode, amp) for b in (b1, b1, b1, b2, b1, b2)]
    plans = model.__dict__.get("_fwd_plans", {})
    assert len(plans) == 1 and next(iter(plans.values())).replays == 5   # recorded on the second call
    for o, r in zip(outs, (ref1, ref1, ref1, ref2, ref1, ref2)):
        assert o.dtype == r.dtype and torch.equal(o, r)
    assert not torch.equal(ref1, ref2)


def test_returned_outputs_are_not_overwritten():
    """The module API returns a copy: an output kept from one call survives the next replay."""
    from alignn_mi355x.synthetic import mp_like_batch
    model = _model()
    b1, b2 = mp_like_batch(4).to(DEV), mp_like_batch(4, first=50).to(DEV)
    ref = _eager(model, b1)
    _planned(model, b1)
    kept = _planned(model, b1)          # a replay
    _planned(model, b2)                 # the next replay writes the plan's output buffer
    assert torch.equal(kept, ref)


def test_other_signature_runs_eager_then_its_own_plan():
    from alignn_mi355x.synthetic import mp_like_batch
    model = _model()
    a, b = mp_like_batch(4).to(DEV), mp_like_batch(6).to(DEV)
    ra, rb = _eager(model, a), _eager(model, b)
    for x, r in ((a, ra), (b, rb), (a, ra), (b, rb), (a, ra), (b, rb)):
        assert torch.equal(_planned(model, x), r)
    assert len(model.__dict__["_fwd_plans"]) == 2


def test_training_mode_and_grad_stay_eager():
    """Dropout / autograd calls never take a plan (only no-grad eval forwards do)."""
    from alignn_mi355x.synthetic import mp_like_batch
    model = _model()
    b = mp_like_batch(4).to(DEV)
    with torch.no_grad():
        model(b)
        model(b)
    n = len(model.__dict__.get("_fwd_plans", {}))
    m, lv = model(b)                    # eval, grad enabled: autograd path
    (m.sum() + lv.sum()).backward()
    model.train()
    with torch.no_grad():
        model(b)
        model(b)
    assert len(model.__dict__.get("_fwd_plans", {})) == n
    assert model.base.node_encoder[0].weight.grad is not None


def test_ensemble_members_replay_bitwise():
    import alignn_mi355x as A
    from alignn_mi355x import infer
    from alignn_mi355x.ensemble import EnsemblePredictor
    from alignn_mi355x.synthetic import mp_like_batch
    models = [_model(seed=s) for s in range(3)]
    batches = [mp_like_batch(8, first=10 * i).to(DEV) for i in range(3)]
    ep = EnsemblePredictor(models)
    infer.ENABLED = False
    try:
        ref = [ep.member_outputs(b).clone() for b in batches]
    finally:
        infer.ENABLED = True
    for _ in range(2):
        got = [ep.member_outputs(b).clone() for b in batches]
        torch.cuda.synchronize()
        for g, r in zip(got, ref):
            assert torch.equal(g, r)
    assert all(len(m.__dict__["_fwd_plans"]) == 1 for m in models)
    assert isinstance(A.infer.ForwardPlan, type)


def test_knn_embeddings_replay_bitwise():
    from alignn_mi355x import infer, knn
    from alignn_mi355x.synthetic import mp_like_batch
    model = _model()
    batches = []
    for i in range(3):
        b = mp_like_batch(4, first=4 * i).to(DEV)
        b.train_idx = torch.arange(4 * i, 4 * i + 4)
        batches.append(b)
    infer.ENABLED = False
    try:
        z0, y0, i0 = knn.embed_collect(model, batches)
        z0 = z0.clone()
    finally:
        infer.ENABLED = True
    knn.embed_collect(model, batches)
    z1, y1, i1 = knn.embed_collect(model, batches)
    assert torch.equal(z1, z0) and torch.equal(y1, y0) and np.array_equal(i1, i0)


@pytest.mark.parametrize("use_graph", [False, True])
def test_graph_and_plan_replay_equal(use_graph):
    """A recorded forward replays as the native plan or as the HIP graph of the same capture (the
    faster one is chosen when it is recorded): both bitwise the eager forward."""
    from alignn_mi355x.synthetic import mp_like_batch
    model = _model()
    b1, b2 = mp_like_batch(6).to(DEV), mp_like_batch(6, first=30).to(DEV)
    ref1, ref2 = _eager(model, b1), _eager(model, b2)
    _planned(model, b1)
    _planned(model, b1)                       # recorded here
    p = next(iter(model.__dict__["_fwd_plans"].values()))
    p.use_graph = use_graph
    for b, r in ((b2, ref2), (b1, ref1), (b1, ref1), (b2, ref2)):
        assert torch.equal(_planned(model, b), r)


def test_small_forward_single_stream_large_keeps_streams():
    """A forward over fewer line-graph edges than infer.SINGLE_STREAM_MAX_T is recorded on one stream
    and may replay as a HIP graph; a larger one keeps the side streams and always replays the native
    plan (a multi-branch graph's runtime-created streams moved later streams' hardware queues).  Both
    bitwise the eager forward, which runs on the side streams either way."""
    from alignn_mi355x import infer
    from alignn_mi355x.synthetic import mp_like_batch
    for nb, single in ((6, True), (12, False)):
        model = _model()
        b = mp_like_batch(nb).to(DEV)
        assert (int(b.lg_edge_index.size(1)) < infer.SINGLE_STREAM_MAX_T) == single
        ref = _eager(model, b)
        _planned(model, b)
        got = _planned(model, b)                  # recorded here
        p = next(iter(model.__dict__["_fwd_plans"].values()))
        assert p.single == single
        if not single:
            assert not p.use_graph
        assert model._engine.overlap_forward   # restored after the recording
        assert torch.equal(got, ref)
        assert torch.equal(_planned(model, b), ref)


def test_replaced_parameter_invalidates_recorded_forward():
    """A parameter replaced after the forward was recorded re-lays the flat buffer out
    (model._ensure_flat): the recorded plans, which read the old buffer, are released and the call
    equals the eager forward with the new weights."""
    from alignn_mi355x.synthetic import mp_like_batch
    model = _model()
    b = mp_like_batch(4).to(DEV)
    _planned(model, b)
    _planned(model, b)
    assert len(model.__dict__["_fwd_plans"]) == 1
    lin = model.base.node_encoder[0]
    g = torch.Generator(device="cpu").manual_seed(3)
    lin.weight = torch.nn.Parameter((torch.randn(lin.weight.shape, generator=g) * 0.05).to(DEV))
    ref = _eager(model, b)
    got = _planned(model, b)
    assert torch.equal(got, ref)
    assert len(model.__dict__.get("_fwd_plans", {})) == 0
