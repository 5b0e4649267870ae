"""Variable-size batches at plan speed (store.BatchCapacity): batches of variable-size MP-like
graphs (8-60 atoms, 2-6 neighbour shells) padded to one capacity by an inert ghost graph all share
one plan signature.  The padded step equals the unpadded step of the same graphs (the reference's
loop body on that batch, train.py:639-699) within fp32 summation-order differences — dropout masks
included, since every real element keeps its position — and a plan captured on one padded batch,
re-bound to others, equals the eager step on each bit for bit with no eager steps."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
KEYS = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y")
_ST = {}


def _store(n=96):
    from alignn_mi355x.data import Data
    from alignn_mi355x.store import GraphStore
    from alignn_mi355x.synthetic import variable_mp_like_graph
    if n not in _ST:
        _ST[n] = GraphStore.from_data_list([Data(**{k: getattr(variable_mp_like_graph(g), k) for k in KEYS})
                                            for g in range(n)], DEV)
    return _ST[n]


def _trainer(dropout=0.15):
    import alignn_mi355x as A
    torch.manual_seed(0)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 256, 4, 4, dropout), 2).to(DEV)
    return A.FusedTrainer(model)


def test_padded_batch_structure():
    from alignn_mi355x.engine import prepare_batch
    st = _store()
    cap = st.capacity(8)
    assert cap.active is not None
    idx = np.random.default_rng(0).choice(st.num_graphs, size=8, replace=False)
    b = st.collate(idx, capacity=cap)
    sz = st.batch_sizes(idx)
    assert b.num_real_graphs == 8 and b.num_graphs == 9
    assert b.x.shape[0] == cap.nodes and b.edge_index.shape[1] == cap.edges and b.lg_edge_index.shape[1] == cap.triplets
    assert b.ptr.numel() == 10 and int(b.ptr[-2]) == sz["nodes"] and int(b.ptr[-1]) == cap.nodes
    assert b.global_x.shape[0] == 59 * 9 and b.y.numel() == 2 * 9
    ei = b.edge_index.cpu()
    assert int(ei[:, sz["edges"]:].min()) >= sz["nodes"] and int(ei.max()) < cap.nodes   # ghost bonds: ghost atoms
    assert int(b.lg_edge_index[:, sz["triplets"]:].min()) >= sz["edges"]
    assert torch.equal(b.batch[sz["nodes"]:].cpu(), torch.full((cap.nodes - sz["nodes"],), 8))
    assert float(b.x[sz["nodes"]:].abs().sum()) == 0.0 and torch.all(b.y[16:] == 1.0)
    bc = prepare_batch(b)
    assert bc.lg.n == cap.active and bc.lg.schedule().n_heavy == 0 and bc.ag.schedule().n_heavy == 0
    # the real part of the padded batch is the unpadded batch
    u = st.collate(idx)
    for k in ("x", "edge_attr", "lg_edge_attr"):
        assert torch.equal(getattr(b, k)[:getattr(u, k).shape[0]], getattr(u, k)), k
    for k in ("edge_index", "lg_edge_index"):
        assert torch.equal(getattr(b, k)[:, :getattr(u, k).shape[1]], getattr(u, k)), k


def test_padded_step_matches_unpadded_step():
    """Same graphs, same seeds (dropout and jitter on): loss and every gradient of the padded step
    within 1e-5 (normwise) of the unpadded step's."""
    from alignn_mi355x.layout import offsets
    st = _store()
    cap = st.capacity(8)
    idx = np.random.default_rng(1).choice(st.num_graphs, size=8, replace=False)
    t1, t2 = _trainer(), _trainer()
    l1 = t1.forward_backward(st.collate(idx), 77).clone()
    l2 = t2.forward_backward(st.collate(idx, capacity=cap), 77).clone()
    torch.cuda.synchronize()
    assert abs(float(l1) - float(l2)) <= 1e-5 * abs(float(l1)), (float(l1), float(l2))
    offs, _, _ = offsets(t1.model.config, True)
    g1, g2 = t1.st.grad.double(), t2.st.grad.double()
    top = max(float(g1[o:o + int(np.prod(sh))].norm()) for o, sh in offs.values())
    checked = 0
    for k, (o, shape) in offs.items():
        n = int(np.prod(shape))
        a, b = g1[o:o + n], g2[o:o + n]
        # parameters whose gradient is ~0 in exact arithmetic (the key biases: a constant shift of every
        # key of a target cancels in its softmax) hold only rounding noise: bounded against the largest
        if float(a.norm()) < 1e-3 * top:
            assert float((a - b).norm()) < 1e-7 * top, k
            continue
        assert float((a - b).norm() / a.norm()) < 1e-5, k
        checked += 1
    assert checked > 50 and float(g2.norm()) > 0


def test_variable_batches_replay_one_plan_bitwise():
    from alignn_mi355x import ops
    from alignn_mi355x.engine import prepare_batch
    st = _store()
    cap = st.capacity(8)
    rng = np.random.default_rng(2)
    te, tp = _trainer(), _trainer()
    tp.capture(st.collate(rng.choice(st.num_graphs, size=8, replace=False), capacity=cap))
    loader = torch.cuda.Stream()
    real = set()
    for i in range(5):
        idx = rng.choice(st.num_graphs, size=8, replace=False)
        real.add(st.batch_sizes(idx)["nodes"])
        with torch.cuda.stream(loader):
            b = st.collate(idx, capacity=cap)
        prepare_batch(b, loader)
        s = 300 + i
        lp = tp.step(b, seed=s).clone()
        te.use_step_seed(tp._seed_dev)
        tp._seed_dev.fill_(s)
        le = te.forward_backward(b, 0).clone()
        te._clip_and_update()
        torch.cuda.synchronize()
        assert torch.equal(le, lp), i
        assert torch.equal(te.st.flat, tp.st.flat), i
    assert len(real) > 1                                   # batches of different real sizes
    assert tp.rebinds == 5 and tp.rebind_misses == 0
    tp.release_capture()
    ops.set_step_seed(None)

