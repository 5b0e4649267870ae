"""Row f2, host side: the oracle's restatement of PtGraphDataset (validity filter,
node-dimension rules, z-scoring, train-only statistics; oracle/dataset_ref.py) reproduces what the
reference's own classes wrote into tests/golden/dataset.npz, bit for bit; a host-side GraphStore
applies the same validity filter and node-dimension rules."""
import numpy as np
import pytest
import torch

from _golden_util import DATASET_MODES, dataset_graphs, dataset_stats
from conftest import load_golden


@pytest.fixture(scope="module")
def z():
    return load_golden("dataset")


@pytest.mark.parametrize("mode", list(DATASET_MODES))
def test_oracle_items_match_reference(z, mode):
    from oracle import dataset_ref
    graphs = dataset_graphs(z)
    kept = [g for g, d in enumerate(graphs) if d["y"] is not None and dataset_ref.is_valid(d)]
    assert kept == list(z[f"{mode}/kept"])
    st = dataset_stats(z, mode)
    xs, gs = zip(*[dataset_ref.item(graphs[g], 206, stats=st, **DATASET_MODES[mode]) for g in kept])
    assert np.array_equal(torch.cat(xs).numpy(), z[f"{mode}/x"])
    assert np.array_equal(torch.stack([g.reshape(-1) for g in gs]).numpy(), z[f"{mode}/global_x"])


def test_oracle_feature_stats_match_reference(z):
    from oracle import dataset_ref
    graphs = dataset_graphs(z)
    kept = [g for g, d in enumerate(graphs) if d["y"] is not None and dataset_ref.is_valid(d)]
    st = dataset_ref.feature_stats([graphs[g] for g in kept], list(z["setup/train_idx"]), 206)
    for k, v in st.items():
        assert np.array_equal(v.numpy(), z[f"setup/stats/{k}"]), k


@pytest.mark.parametrize("mode", list(DATASET_MODES))
def test_host_store_filter_and_node_dims(z, mode):
    from alignn_mi355x.data import Data
    from alignn_mi355x.store import GraphStore
    graphs = dataset_graphs(z)
    st = GraphStore.from_data_list([Data(**d) for d in graphs], "cpu", **DATASET_MODES[mode])
    kept = [g for g in range(len(graphs)) if graphs[g]["y"] is not None]   # no-target graph skipped first
    assert [kept[i] for i in st.ids] == list(z[f"{mode}/kept"])
    if f"{mode}/node_dim" in z:
        assert st.node_dim == int(z[f"{mode}/node_dim"])
    with pytest.raises(ValueError):
        GraphStore.from_data_list([Data(**d) for d in graphs], "cpu", force_node_dim=3)
