"""Row f2 on the device: a GraphStore built from the raw graphs of
tests/golden/dataset.npz drops the same invalid graphs on the device (NaN / inf in any float field,
no target) and its collate — PtGraphDataset.__getitem__'s select / pad / truncate and z-scoring fused
into the copy kernel — equals what the reference's own PtGraphDataset returned, bit for bit, in every
mode (use_mat2vec, force_node_dim truncate / pad, the reference's _setup statistics and the shipped
ensemble's scaler_state.pt).  The device statistics (fp64 per-graph sums in train_idx order) equal
the reference's _setup statistics; a standardized batch trains through the engine."""
import numpy as np
import pytest
import torch

from _golden_util import DATASET_MODES, dataset_graphs, dataset_stats
from conftest import load_golden

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _store(z, mode):
    from alignn_mi355x.data import Data
    from alignn_mi355x.store import GraphStore
    return GraphStore.from_data_list([Data(**d) for d in dataset_graphs(z)], DEV, **DATASET_MODES[mode])


@pytest.mark.parametrize("mode", list(DATASET_MODES))
def test_store_collate_matches_reference_dataset(mode):
    z = load_golden("dataset")
    st = _store(z, mode)
    assert st.num_graphs == len(z[f"{mode}/kept"])
    st.set_feature_standardization(**dataset_stats(z, mode))
    n = st.num_graphs
    b = st.collate(np.arange(n))
    torch.cuda.synchronize()
    assert np.array_equal(b.x.cpu().numpy(), z[f"{mode}/x"])
    assert np.array_equal(b.global_x.cpu().numpy().reshape(n, -1), z[f"{mode}/global_x"])
    assert torch.equal(b.sample_index.cpu(), torch.arange(n))
    # a shuffled sub-batch is the same rows in batch order
    sel = np.array([3, 0, n - 1, 7])
    bs = st.collate(sel)
    rows = np.split(z[f"{mode}/x"], np.cumsum(st.counts["x"][st.ids])[:-1])
    assert np.array_equal(bs.x.cpu().numpy(), np.concatenate([rows[i] for i in sel]))
    # statistics removed again: raw selection / padding only
    st.set_feature_standardization()
    raw = st.collate(np.arange(n)).x.cpu().numpy()
    assert raw.shape == z[f"{mode}/x"].shape and not np.array_equal(raw, z[f"{mode}/x"])


def test_device_feature_stats_match_reference_setup():
    z = load_golden("dataset")
    st = _store(z, "setup")
    got = st.feature_stats(list(z["setup/train_idx"]))
    for k, v in got.items():
        want = z[f"setup/stats/{k}"]
        assert v is not None and v.dtype == torch.float32, k
        # fp64 sums in another association than torch's CPU reduction: equal after the fp32 rounding
        # except (rarely) one ulp
        np.testing.assert_allclose(v.numpy(), want, rtol=1.2e-7, atol=0, err_msg=k)


def test_standardized_store_batch_trains():
    """The 206-wide standardized batch of the store through the fused training step (engine dims:
    node 206, global 59 + 230): finite loss and gradients."""
    import alignn_mi355x as A
    z = load_golden("dataset")
    st = _store(z, "shipped")
    st.set_feature_standardization(**dataset_stats(z, "shipped"))
    torch.manual_seed(0)
    model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 64, 2, 4, 0.0), 2).to(DEV)
    tr = A.FusedTrainer(model)
    b = st.collate(np.arange(8))
    loss = tr.forward_backward(b, 3).clone()
    torch.cuda.synchronize()
    assert torch.isfinite(loss).all() and torch.isfinite(tr.st.grad).all()
