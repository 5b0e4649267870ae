"""Host-side guards added in round 4 (no GPU): the padded batch's compaction fill, the collated
line-graph index bound behind a store batch's trusted flag, and a replay refusing a gradient exchange
that changed after capture."""
import weakref

import numpy as np
import pytest
import torch


def test_fill_active_takes_unused_ghost_bonds_first_then_inert_bonds():
    """BatchCache._fill_active marks exactly na bonds: ghost bonds past `first` in index order, then —
    when the real active count is below the host bound and the ghost room is short — real inactive
    bonds (no line-graph edges: empty segments, never sources).  Before round 4 only ghost bonds were
    taken, so the compaction's nonzero_static list was padded with -1 (engine.py:275)."""
    from alignn_mi355x.engine import BatchCache
    n, first = 20, 16
    active = torch.zeros(n, dtype=torch.bool)
    active[[1, 2, 5, 9, 16]] = True          # real active bonds, and 16: already marked
    out = BatchCache._fill_active(active.clone(), first, 8)
    assert int(out.sum()) == 8
    assert out[[1, 2, 5, 9, 16]].all()
    assert out[17:20].all()                   # the unused ghost bonds first
    assert int(out[:first].sum()) == 4        # no real bond needed yet
    out = BatchCache._fill_active(active.clone(), first, 12)   # ghost room (3) short by 4
    assert int(out.sum()) == 12
    assert out[17:20].all()
    assert out[[0, 3, 4, 6]].all() and not out[[7, 8, 10]].any()   # the lowest inactive real bonds next
    out = BatchCache._fill_active(active.clone(), first, 5)    # nothing to add
    assert torch.equal(out, active)
    rows = torch.nonzero_static(BatchCache._fill_active(active.clone(), first, 12), size=12).flatten()
    assert int(rows.min()) >= 0


def test_collated_line_graph_index_bound_under_pyg_offsets():
    """GraphStore._lg_bound_ok: with lg_offset='num_nodes' a batch's lg_edge_index (+ the atom-count
    increment) may point past the batch's bonds when a graph has fewer bonds than atoms; such a batch
    must not skip the per-batch index check (store.py:575)."""
    from alignn_mi355x.data import Data
    from alignn_mi355x.store import GraphStore
    keys = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y")

    def graph(n_atoms, bonds, lg_hi):
        ei = torch.stack([torch.arange(bonds) % n_atoms, (torch.arange(bonds) + 1) % n_atoms])
        lg = torch.tensor([[0, lg_hi], [lg_hi, 0]])
        return Data(x=torch.zeros(n_atoms, 4), edge_index=ei, edge_attr=torch.zeros(bonds, 2),
                    lg_edge_index=lg, lg_edge_attr=torch.zeros(2, 3), global_x=torch.zeros(59, 1),
                    sg_one_hot=torch.zeros(230, 1), y=torch.ones(2))

    # graph 0: 10 atoms, 4 bonds (fewer bonds than atoms); graph 1: 2 atoms, 6 bonds touching bond 5
    st = GraphStore.from_data_list([Data(**{k: getattr(g, k) for k in keys})
                                    for g in (graph(10, 4, 3), graph(2, 6, 5))], "cpu")
    assert st.indices_checked                                   # each graph is fine on its own
    # order (0, 1): graph 1's bond 5 + 10 atoms = 15 >= 10 bonds in the batch
    assert not st._lg_bound_ok(np.array([0, 1]), "num_nodes")
    assert st._lg_bound_ok(np.array([1, 0]), "num_nodes")       # 3 + 2 = 5 < 10
    assert st._lg_bound_ok(np.array([0, 1]), "num_edges")       # implied by the bond increments


class _ReplayLib:
    def alignn_set_i64(self, *a):
        return 0

    def alignn_plan_replay(self, *a):
        return 0


class _Slot:
    """A captured batch stand-in (weak-referenceable, no tensors)."""


def test_replay_refuses_exchange_changed_after_capture(monkeypatch):
    """The phases of a captured step are cut for the exchange in place at capture (grad_buckets: three
    phases, a hook or none: two); a replay after grad_buckets / grad_hook changed raises instead of
    skipping the all_reduce or crashing (trainer.py:356)."""
    import alignn_mi355x as A
    from alignn_mi355x import _lib, ops, trainer as trainer_mod
    from alignn_mi355x.engine import batch_versions
    torch.manual_seed(0)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(6, 8, 7, 289, 2, 32, 1, 1, 0.0), 2)
    tr = A.FusedTrainer(model, optimizer="torch")
    monkeypatch.setattr(_lib, "lib", lambda: _ReplayLib())
    monkeypatch.setattr(ops, "stream_ptr", lambda *a, **k: 0)
    monkeypatch.setattr(trainer_mod, "check", lambda rc, what: None)
    tr._seed_dev = torch.zeros(1, dtype=torch.int64)
    batch = _Slot()
    calls = []
    tr.grad_hook = lambda g: calls.append(1)
    tr._graph = (None, None, batch, [1, 2])
    tr._bound, tr._bound_v = weakref.ref(batch), batch_versions(batch, trainer_mod.BATCH_FIELDS)
    tr._exchange = tr._exchange_mode()
    tr.step(batch, seed=1)
    assert calls == [1]
    tr.grad_hook = None
    with pytest.raises(RuntimeError, match="exchange changed after capture"):
        tr.step(batch, seed=2)
    tr.grad_hook = lambda g: calls.append(2)   # a different hook object is a different exchange
    with pytest.raises(RuntimeError, match="exchange changed after capture"):
        tr.step(batch, seed=3)


@pytest.mark.parametrize("lg_offset", ["num_nodes", "num_edges"])
def test_store_degree_and_active_bounds_cover_the_collated_batch(lg_offset):
    """GraphStore.degree_bounds / batch_sizes['active'] (the host facts behind a store batch's device-
    built schedules and sync-free compaction): every in-degree of the collated atom and line graphs and
    the line graph's active-bond count lie within them, on graphs of mixed sizes (overlapping PyG
    windows of different widths) — and on MP-like graphs they are exact."""
    from alignn_mi355x.data import Batch
    from alignn_mi355x.store import GraphStore
    from alignn_mi355x.synthetic import mp_like_graph
    sizes = [(60, 6), (24, 3), (40, 5), (13, 2), (60, 6), (31, 4), (9, 1)]
    mixed = [mp_like_graph(g, n_atoms=sizes[g % 7][0], half_degree=sizes[g % 7][1]) for g in range(14)]
    mp = [mp_like_graph(g) for g in range(12)]
    rng = np.random.default_rng(7)
    for gs, exact in ((mixed, False), (mp, True)):
        st = GraphStore.from_data_list(gs, "cpu")
        for _ in range(6):
            sel = rng.choice(len(gs), size=int(rng.integers(1, len(gs))), replace=False)
            b = Batch.from_data_list([gs[i] for i in sel], lg_offset=lg_offset)
            hb = st.degree_bounds(st.ids[sel], lg_offset)
            E = b.edge_index.size(1)
            ag = int(torch.bincount(b.edge_index[1], minlength=b.x.size(0)).max())
            lg = int(torch.bincount(b.lg_edge_index[1], minlength=E).max())
            act = torch.zeros(E, dtype=torch.bool)
            act[b.lg_edge_index[0]] = True
            act[b.lg_edge_index[1]] = True
            bound_act = st.batch_sizes(sel, lg_offset)["active"]
            assert ag <= hb["ag"] and lg <= hb["lg"] and int(act.sum()) <= bound_act, (list(sel), hb)
            if exact:
                assert (ag, lg, int(act.sum())) == (hb["ag"], hb["lg"], bound_act)
