"""HBM-resident dataset + on-device collate vs PyG's collation rules (the oracle's
restatement) — bit-exact — and a training step on a device-collated batch vs the host-collated one.
Sorts after the core suites."""
import numpy as np
import pytest
import torch

from oracle.pyg_ref import RefData, collate

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _graphs(n=7):
    from alignn_mi355x.synthetic import mp_like_graph
    sizes = [(60, 6), (24, 3), (40, 5), (13, 2), (60, 6), (31, 4), (9, 1)]
    return [mp_like_graph(g, n_atoms=sizes[g % len(sizes)][0], half_degree=sizes[g % len(sizes)][1])
            for g in range(n)]


@pytest.mark.parametrize("lg_offset", ["num_nodes", "num_edges"])
def test_device_collate_bit_exact(lg_offset):
    from alignn_mi355x.store import GraphStore
    gs = _graphs()
    st = GraphStore.from_data_list(gs, DEV)
    for sel in ([0, 1, 2, 3, 4, 5, 6], [6, 2, 2, 0], [3]):
        b = st.collate(sel, lg_offset)
        ref = collate([RefData(**{k: getattr(gs[i], k) for k in gs[i].keys()}) for i in sel], lg_offset=lg_offset)
        for k in ("x", "edge_index", "edge_attr", "lg_edge_index", "lg_edge_attr", "global_x", "sg_one_hot", "y",
                  "batch", "ptr"):
            got, want = getattr(b, k).cpu(), getattr(ref, k)
            assert got.shape == want.shape and torch.equal(got, want.to(got.dtype)), (k, sel)
        assert b.num_graphs == len(sel)


def test_train_step_on_store_batch_equals_host_batch():
    import alignn_mi355x as A
    from alignn_mi355x.store import GraphStore
    from alignn_mi355x.synthetic import mp_like_graph
    gs = [mp_like_graph(g) for g in range(6)]
    st = GraphStore.from_data_list(gs, DEV)
    sel = [4, 1, 3]
    b_dev = st.collate(sel)
    b_host = A.Batch.from_data_list([gs[i] for i in sel]).to(DEV)
    grads = []
    for b in (b_dev, b_host):
        torch.manual_seed(0)
        model = A.HeteroAlignnRegressor(A.AlignnRegressor(206, 36, 11, 289, 2, 64, 2, 4, 0.15), 2).to(DEV)
        tr = A.FusedTrainer(model)
        tr.forward_backward(b, 5)
        grads.append(tr.st.grad.clone())
    torch.cuda.synchronize()
    assert torch.equal(grads[0], grads[1])


def test_copy_many_one_launch_matches_torch_copies():
    """alignn_copy_many (re-binding a captured step: batch fields + device cache in one launch):
    mixed dtypes, sizes with a partial last 16-byte unit, more than 32 pairs (two launches), and
    pairs the kernel does not take (non-contiguous) through torch's copy."""
    import torch
    from alignn_mi355x import ops
    g = torch.Generator(device="cpu").manual_seed(3)
    pairs, refs = [], []
    for i in range(45):
        n = int(torch.randint(1, 5000, (1,), generator=g))
        dt = (torch.float32, torch.int32, torch.int64)[i % 3]
        src = (torch.randn(n, generator=g) * 1000).to(dt).to("cuda")
        dst = torch.zeros_like(src)
        pairs.append((dst, src))
        refs.append(src.clone())
    big = torch.randn(300, 7, generator=g).to("cuda")
    nc_dst = torch.zeros(7, 300, device="cuda").t()          # non-contiguous destination: torch fallback
    pairs.append((nc_dst, big))
    ops.copy_many(pairs)
    torch.cuda.synchronize()
    for (dst, _), ref in zip(pairs[:-1], refs):
        assert torch.equal(dst, ref)
    assert torch.equal(nc_dst, big)
