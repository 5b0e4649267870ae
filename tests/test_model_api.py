"""Drop-in API checks on CPU: constructor signatures/ValueErrors, state-dict keys identical to the
reference's (golden fixtures were written from the reference's own modules), flat layout,
PyG-compatible collation.  No GPU."""
import pytest
import torch

import alignn_mi355x as A
from alignn_mi355x.layout import AlignnConfig, offsets
from alignn_mi355x.synthetic import mp_like_graph
from oracle.pyg_ref import RefData, collate


def _model(hidden=64, layers=2, heads=4, node=206, edge=36, angle=11):
    base = A.AlignnRegressor(node, edge, angle, 289, 2, hidden, layers, heads, 0.0)
    return A.HeteroAlignnRegressor(base, 2)


@pytest.mark.parametrize("case", ["mp_d64_quirk", "smoke_c1"])
def test_state_dict_keys_and_shapes_match_reference(golden, case):
    g = golden(case)
    ref = {k[2:]: v.shape for k, v in g.items() if k.startswith("p/")}
    meta = {k[5:]: int(g[k]) for k in g if k.startswith("meta/") and g[k].ndim == 0}
    base = A.AlignnRegressor(meta["node"], meta["edge"], meta["angle"], meta["global"], 2, meta["hidden"],
                             meta["layers"], meta["heads"], 0.0)
    m = A.HeteroAlignnRegressor(base, 2)
    sd = m.state_dict()
    assert list(sd.keys()) == list(ref.keys())
    for k, v in sd.items():
        assert tuple(v.shape) == tuple(ref[k]), k
    m.load_state_dict({k: torch.from_numpy(g["p/" + k]) for k in ref})


def test_full_size_param_count():
    m = _model(256, 4, 4)
    assert sum(p.numel() for p in m.parameters()) == 3307270
    assert len(m.state_dict()) == 130


def test_value_errors():
    with pytest.raises(ValueError):
        A.AlignnRegressor(6, 8, 7, 289, 2, 30, 1, 4, 0.0)
    with pytest.raises(ValueError):
        A.AlignnRegressor(6, 8, 7, 289, 2, 32, 1, 0, 0.0)
    with pytest.raises(ValueError):
        A.AlignnRegressor(6, 8, 7, 289, 0, 32, 1, 1, 0.0)
    with pytest.raises(ValueError):
        A.EdgeUpdateBlock(30, 4, 0.1)
    with pytest.raises(ValueError):
        A.NodeUpdateBlock(30, 30, 4, 0.1)


def test_layout_covers_every_trainable_parameter_once():
    cfg = AlignnConfig(206, 36, 11, 289, 2, 64, 2, 4, 0.0)
    offs, total, sigma = offsets(cfg, True)
    m = _model()
    named = dict(m.named_parameters())
    trainable = {k for k in named if not k.startswith("base.output_heads.")}
    assert set(offs) == trainable
    assert total == sum(named[k].numel() for k in trainable)
    ends = sorted((o, o + named[k].numel()) for k, (o, _) in offs.items())
    for (a0, a1), (b0, _) in zip(ends, ends[1:]):
        assert a1 == b0
    assert all(o >= sigma for k, (o, _) in offs.items() if k.startswith("logvar_heads."))
    assert all(o < sigma for k, (o, _) in offs.items() if not k.startswith("logvar_heads."))


def test_cpu_forward_fails_loudly():
    m = _model()
    b = A.Batch.from_data_list([mp_like_graph(0)])
    with pytest.raises(RuntimeError, match="HIP device"):
        m(b)


@pytest.mark.parametrize("mode", ["num_nodes", "num_edges"])
def test_collate_matches_oracle(mode):
    gs = [mp_like_graph(g) for g in range(3)]
    b = A.Batch.from_data_list(gs, lg_offset=mode)
    r = collate([RefData(**{k: getattr(d, k) for k in d.keys()}) for d in gs], lg_offset=mode)
    for k in ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y",
              "batch", "ptr"):
        assert torch.equal(getattr(b, k), getattr(r, k)), k
    assert b.num_graphs == 3


def test_tconv_host_shape_checks_reject_undersized_operands():
    """The attention wrappers refuse (ValueError) operands smaller than the graph before any launch."""
    import types
    from alignn_mi355x import ops
    g = types.SimpleNamespace(n=10, m=40)
    D, H = 64, 4
    ok = dict(QKVR=torch.zeros(10, 3 * D), F=torch.zeros(40, D))
    ops._check_tconv(g, D, H, ok["QKVR"], ok["F"], None)
    with pytest.raises(ValueError):
        ops._check_tconv(g, D, H, ok["QKVR"], torch.zeros(39, D), None)     # F short of m rows
    with pytest.raises(ValueError):
        ops._check_tconv(g, D, H, torch.zeros(9, 3 * D), ok["F"], None)     # QKVR short of n rows
    with pytest.raises(ValueError):
        ops._check_tconv(g, D, H, ok["QKVR"], None, None)                    # no edge features
    with pytest.raises(ValueError):
        ops._check_tconv(g, D, H, ok["QKVR"], ok["F"], None, edge_heads=(torch.zeros(40, 3),))


def test_mp_like_line_graph_is_the_per_graph_construction():
    """synthetic._circulant computes the line graph once: it equals the per-graph construction
    (fetch.py:419-447 order) on the permuted bond list for any seed (SURVEY §8d generator)."""
    import numpy as np
    from alignn_mi355x import synthetic as S
    for g in (0, 3, 1234):
        d = mp_like_graph(g)
        src, dst = d.edge_index.numpy()
        ls, ld = S._line_graph(src, dst)
        assert np.array_equal(ls, d.lg_edge_index[0].numpy()) and np.array_equal(ld, d.lg_edge_index[1].numpy())
        assert d.lg_edge_index.size(1) == 7920 and d.edge_index.size(1) == 720
