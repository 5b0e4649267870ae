"""HBM-resident dataset, host side: the collate plan (starts, counts, PyG increments)
applied by a numpy emulation of the device kernels reproduces the oracle's restatement of PyG's
Batch.from_data_list bit for bit, in both lg_offset modes; save/load round-trips without pickles."""
import numpy as np
import pytest
import torch

from oracle.pyg_ref import RefData, collate


def _graphs(n=7):
    """Ragged MP-like graphs (different atom counts and degrees), plus one spare entry."""
    from alignn_mi355x.synthetic import mp_like_graph
    sizes = [(60, 6), (24, 3), (40, 5), (13, 2), (60, 6), (31, 4), (9, 1)]
    return [mp_like_graph(g, n_atoms=sizes[g % len(sizes)][0], half_degree=sizes[g % len(sizes)][1])
            for g in range(n)]


@pytest.mark.parametrize("lg_offset", ["num_nodes", "num_edges"])
def test_plan_matches_pyg_collate(lg_offset):
    from alignn_mi355x.store import CollatePlan, GraphStore, _excl_cumsum
    gs = _graphs()
    # the smoke graph has other feature widths: build two stores (MP-like / smoke) like real data would
    mp = gs[:-1]
    arrays, counts, meta, _ = GraphStore.host_arrays(mp)
    starts = {f: _excl_cumsum(c) for f, c in counts.items()}
    for sel in ([0, 1, 2], [5, 0, 3, 3], [4]):
        pl = CollatePlan(meta, counts, starts, np.asarray(sel), lg_offset)
        got = pl.apply_host(arrays, meta)
        ref = collate([RefData(**{k: getattr(mp[i], k) for k in mp[i].keys()}) for i in sel], lg_offset=lg_offset)
        for k in meta:
            want = getattr(ref, k).numpy()
            g = got[k].reshape(want.shape) if meta[k]["kind"] == "rows" else got[k]
            assert g.dtype == want.dtype or meta[k]["kind"] == "rows", k
            assert np.array_equal(g, want), (k, sel)
        assert np.array_equal(got["batch"], ref.batch.numpy())
        assert np.array_equal(got["ptr"], ref.ptr.numpy())


def test_store_save_load_roundtrip(tmp_path):
    from alignn_mi355x.store import GraphStore
    gs = _graphs(4)[:-1]
    st = GraphStore.from_data_list(gs, "cpu")
    st.save(str(tmp_path / "ds"))
    st2 = GraphStore.load(str(tmp_path / "ds"), "cpu")
    assert st2.meta == st.meta and st2.num_graphs == 3
    for k in st.arrays:
        assert torch.equal(st.arrays[k], st2.arrays[k]), k
        assert np.array_equal(st.counts[k], st2.counts[k]), k


def test_plan_rejects_bad_indices():
    from alignn_mi355x.store import GraphStore
    st = GraphStore.from_data_list(_graphs(3)[:-1], "cpu")
    with pytest.raises(IndexError):
        st.plan([0, 5])
    with pytest.raises(ValueError):
        st.plan([])
    with pytest.raises(ValueError):
        st.plan([0], lg_offset="bogus")


def test_index_ranges_checked_once_at_build():
    """GraphStore checks every stored graph's edge_index / lg_edge_index against its own atom / bond
    counts once (so collated batches skip the per-batch check); a graph pointing outside itself
    leaves the store unchecked, and batches are then validated as PyG would at use."""
    from alignn_mi355x.data import Data
    from alignn_mi355x.store import GraphStore
    keys = ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y")
    gs = [Data(**{k: getattr(g, k) for k in keys}) for g in _graphs(4)]
    assert GraphStore.from_data_list(gs, "cpu").indices_checked
    bad = [Data(**{k: getattr(g, k).clone() for k in keys}) for g in _graphs(4)]
    bad[2].edge_index[1, 3] = bad[2].x.size(0)            # one past the graph's atoms
    assert not GraphStore.from_data_list(bad, "cpu").indices_checked
    bad = [Data(**{k: getattr(g, k).clone() for k in keys}) for g in _graphs(4)]
    bad[1].lg_edge_index[0, 0] = bad[1].edge_index.size(1)   # one past the graph's bonds
    assert not GraphStore.from_data_list(bad, "cpu").indices_checked
