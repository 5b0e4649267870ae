"""Fixed-capacity batches (store.BatchCapacity), host side: the ghost plan fits or refuses a batch
by the capacity's sizes and the ghost in-degree bound, the ghost rings stay inside the ghost ids, and
a capacity estimated from random batches of a variable-size store holds them."""
import numpy as np
import pytest


def test_ghost_plan_rules():
    from alignn_mi355x.store import BatchCapacity, ghost_plan, ghost_edges_host
    cap = BatchCapacity(graphs=4, nodes=120, edges=1400, triplets=15000, active=600)
    gp = ghost_plan(cap, 4, 100, 1300, 14000)
    assert gp == {"ga": 20, "ge": 100, "gt": 1000, "kg": 5, "N": 100, "E": 1300, "T": 14000}
    assert ghost_plan(cap, 3, 100, 1300, 14000) is None          # real graph count is part of the capacity
    assert ghost_plan(cap, 4, 120, 1300, 14000) is None          # no room for a ghost atom
    assert ghost_plan(cap, 4, 100, 1401, 14000) is None          # too many bonds
    assert ghost_plan(cap, 4, 119, 1000, 14000) is None          # 400 ghost bonds on 1 ghost atom: in-degree 400
    tight = BatchCapacity(graphs=4, nodes=120, edges=1301, triplets=15000, active=600)
    assert ghost_plan(tight, 4, 100, 1300, 14000) is None        # 1000 ghost triplets on 1 ghost bond
    e = ghost_edges_host(gp["ge"], gp["N"], gp["ga"])
    assert e.shape == (2, 100) and e.min() >= 100 and e.max() < 120
    assert np.bincount(e[1]).max() <= cap.max_in_degree
    t = ghost_edges_host(gp["gt"], gp["E"], gp["kg"])
    assert t.min() >= 1300 and t.max() < 1305 and np.bincount(t[1] - 1300).max() <= cap.max_in_degree


@pytest.mark.parametrize("lg_offset", ["num_nodes", "num_edges"])
def test_capacity_holds_random_batches(lg_offset):
    from alignn_mi355x.data import Data
    from alignn_mi355x.store import GraphStore
    from alignn_mi355x.synthetic import variable_mp_like_graph
    keys = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y")
    gs = [variable_mp_like_graph(g, node_dim=8, edge_dim=4, angle_dim=3) for g in range(60)]
    st = GraphStore.from_data_list([Data(**{k: getattr(d, k) for k in keys}) for d in gs], "cpu")
    assert len({int(d.x.size(0)) for d in gs}) > 10                   # really variable sizes
    cap = st.capacity(8, lg_offset, samples=200)
    assert (cap.active is not None) == (lg_offset == "num_nodes")     # PyG offset rule: compacted line graph
    rng = np.random.default_rng(1)
    fits = 0
    for _ in range(100):
        idx = rng.choice(60, size=8, replace=False)
        if st.fits(idx, cap, lg_offset) is not None:
            fits += 1
    assert fits >= 95, fits
    # the active-bond bound is exact for graphs whose every bond has line-graph edges
    idx = np.arange(8)
    from oracle.pyg_ref import RefData, collate
    ref = collate([RefData(**{k: getattr(gs[i], k) for k in keys}) for i in idx], lg_offset=lg_offset)
    assert st.batch_sizes(idx, lg_offset)["active"] == int(np.unique(ref.lg_edge_index.numpy()).size)
