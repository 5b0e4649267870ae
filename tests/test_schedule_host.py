"""Attention work lists (ops.schedule_lists, the vectorised host schedule): identical to the
straightforward per-range construction they replace, for ragged degree mixes, every chunk size and
with / without the XCD ranges; a permutation of the light targets plus the heavy ones."""
import numpy as np
import pytest
import torch


def _reference(deg, thr, by_degree, xcd, xcds, chunk):
    deg_t = torch.from_numpy(deg)
    n = len(deg)
    heavy_mask = deg_t > thr
    idx = torch.arange(n, dtype=torch.int64)
    light_mask = ~heavy_mask
    lit = idx[light_mask & (deg_t > 0)]
    hv = idx[heavy_mask]
    if by_degree:
        lit = lit[torch.sort(deg_t[lit], descending=True, stable=True).indices]
        hv = hv[torch.sort(deg_t[hv], descending=True, stable=True).indices]
    if xcd and lit.numel() > xcds:
        cum = torch.cumsum(deg_t, 0)
        tot = int(cum[-1])
        bounds = [0] + [int(torch.searchsorted(cum, tot * x // xcds, right=True)) for x in range(1, xcds)] + [n]
        parts = []
        for x in range(xcds):
            sel = lit[(lit >= bounds[x]) & (lit < bounds[x + 1])]
            parts.append(sel[torch.sort(deg_t[sel], descending=True, stable=True).indices].tolist())
        order, j = [], 0
        while any(j * chunk < len(q) for q in parts):
            for q in parts:
                order += q[j * chunk:(j + 1) * chunk]
            j += 1
        lit = torch.tensor(order, dtype=torch.int64)
    return torch.cat([lit, idx[light_mask & (deg_t == 0)]]).numpy(), hv.numpy()


@pytest.mark.parametrize("chunk", [1, 4, 7])
@pytest.mark.parametrize("xcd", [True, False])
def test_schedule_lists_match_reference(chunk, xcd):
    from alignn_mi355x.ops import schedule_lists
    rng = np.random.default_rng(chunk * 2 + int(xcd))
    cases = [rng.integers(0, 140, 2580), np.r_[np.full(1260, 132), rng.integers(0, 133, 1320)],
             rng.integers(0, 400, 300), np.zeros(20, np.int64), rng.integers(0, 3, 9), np.asarray([5, 0, 300, 1])]
    for deg in cases:
        deg = deg.astype(np.int64)
        got = schedule_lists(deg, 256, True, xcd, 8, chunk)
        want = _reference(deg, 256, True, xcd, 8, chunk)
        assert np.array_equal(got[0], want[0]) and np.array_equal(got[1], want[1])
        assert sorted(np.r_[got[0], got[1]].tolist()) == list(range(len(deg)))
