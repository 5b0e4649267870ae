"""Known-answer tests for the oracle's PyG 2.7.0 restatement (PyG itself is absent: SURVEY §8c).

The expected values are computed with explicit pure-Python loops straight from the published
TransformerConv / softmax / mean-pool formulas, on a 7-node / 19-edge graph with a zero-in-degree
node and a node of in-degree 6 (SURVEY §8c golden vector (3))."""
import math

import pytest
import torch

from oracle.pyg_ref import RefData, collate, global_mean_pool, segment_softmax, transformer_conv


def _graph():
    g = torch.Generator().manual_seed(7)
    n, D, H = 7, 8, 2
    # node 0 has no in-edges, node 3 has in-degree 6
    dst = [3, 3, 3, 3, 3, 3, 1, 1, 2, 4, 4, 5, 5, 5, 6, 6, 2, 1, 6]
    src = [0, 1, 2, 4, 5, 6, 0, 3, 1, 0, 2, 3, 4, 6, 1, 5, 6, 6, 6]
    ei = torch.tensor([src, dst])
    x = torch.randn(n, D, generator=g, dtype=torch.float64)
    ea = torch.randn(len(src), D, generator=g, dtype=torch.float64)
    p = {}
    for name in ("lin_query", "lin_key", "lin_value", "lin_skip"):
        p[f"{name}.weight"] = torch.randn(D, D, generator=g, dtype=torch.float64) * 0.4
        p[f"{name}.bias"] = torch.randn(D, generator=g, dtype=torch.float64) * 0.1
    p["lin_edge.weight"] = torch.randn(D, D, generator=g, dtype=torch.float64) * 0.4
    p["lin_beta.weight"] = torch.randn(1, 3 * D, generator=g, dtype=torch.float64) * 0.3
    return x, ei, ea, p, H


def _loop_conv(x, ei, ea, p, H):
    n, D = x.shape
    C = D // H
    W = {k: v.tolist() for k, v in p.items()}
    X, EA = x.tolist(), ea.tolist()

    def lin(name, v, bias=True):
        w = W[name + ".weight"]
        return [sum(w[o][i] * v[i] for i in range(len(v))) + (W[name + ".bias"][o] if bias else 0.0)
                for o in range(len(w))]

    Q = [lin("lin_query", X[i]) for i in range(n)]
    K = [lin("lin_key", X[i]) for i in range(n)]
    V = [lin("lin_value", X[i]) for i in range(n)]
    E = [lin("lin_edge", EA[t], bias=False) for t in range(len(EA))]
    src, dst = ei[0].tolist(), ei[1].tolist()
    out = [[0.0] * D for _ in range(n)]
    for i in range(n):
        edges = [t for t in range(len(src)) if dst[t] == i]
        for h in range(H):
            zs = []
            for t in edges:
                j = src[t]
                zs.append(sum(Q[i][h * C + c] * (K[j][h * C + c] + E[t][h * C + c]) for c in range(C)) / math.sqrt(C))
            if not zs:
                continue
            m = max(zs)
            ex = [math.exp(z - m) for z in zs]
            s = sum(ex) + 1e-16
            for t, e in zip(edges, ex):
                j = src[t]
                for c in range(C):
                    out[i][h * C + c] += (e / s) * (V[j][h * C + c] + E[t][h * C + c])
    y = []
    for i in range(n):
        r = lin("lin_skip", X[i])
        feat = out[i] + r + [a - b for a, b in zip(out[i], r)]
        logit = sum(W["lin_beta.weight"][0][k] * feat[k] for k in range(3 * D))
        beta = 1.0 / (1.0 + math.exp(-logit))
        y.append([beta * r[k] + (1 - beta) * out[i][k] for k in range(D)])
    return torch.tensor(y, dtype=torch.float64)


def test_transformer_conv_known_answer():
    x, ei, ea, p, H = _graph()
    got = transformer_conv(x, ei, ea, p, H)
    want = _loop_conv(x, ei, ea, p, H)
    assert torch.allclose(got, want, rtol=1e-12, atol=1e-12)
    # the zero-in-degree node gets only the gated skip path: out = beta * x_r with agg = 0
    r0 = x[0] @ p["lin_skip.weight"].T + p["lin_skip.bias"]
    b0 = torch.sigmoid(torch.cat([torch.zeros_like(r0), r0, -r0]) @ p["lin_beta.weight"][0])
    assert torch.allclose(got[0], b0 * r0, rtol=1e-12, atol=1e-12)


def test_transformer_conv_gradcheck():
    x, ei, ea, p, H = _graph()
    x.requires_grad_(True)
    ea.requires_grad_(True)
    w = p["lin_edge.weight"].requires_grad_(True)

    def f(x_, ea_, w_):
        q = dict(p)
        q["lin_edge.weight"] = w_
        return transformer_conv(x_, ei, ea_, q, H)

    assert torch.autograd.gradcheck(f, (x, ea, w), eps=1e-6, atol=1e-7)


def test_segment_softmax_sums_to_one_and_empty_segments():
    z = torch.randn(19, 2, dtype=torch.float64)
    idx = torch.tensor([3] * 6 + [1, 1, 2, 4, 4, 5, 5, 5, 6, 6, 2, 1, 6])
    a = segment_softmax(z, idx, 7)
    sums = torch.zeros(7, 2, dtype=torch.float64).index_add_(0, idx, a)
    assert torch.allclose(sums[1:], torch.ones(6, 2, dtype=torch.float64))
    assert torch.all(sums[0] == 0)


def test_global_mean_pool():
    x = torch.arange(12.0).view(6, 2)
    b = torch.tensor([0, 0, 1, 1, 1, 2])
    want = torch.tensor([[1.0, 2.0], [6.0, 7.0], [10.0, 11.0]])
    assert torch.equal(global_mean_pool(x, b), want)


@pytest.mark.parametrize("mode", ["num_nodes", "num_edges"])
def test_collate_offsets(mode):
    d1 = RefData(x=torch.zeros(3, 1), edge_index=torch.tensor([[0, 1, 2, 0], [1, 2, 0, 2]]),
                 lg_edge_index=torch.tensor([[0, 1], [1, 2]]), y=torch.ones(2))
    d2 = RefData(x=torch.zeros(2, 1), edge_index=torch.tensor([[0, 1], [1, 0]]),
                 lg_edge_index=torch.tensor([[0], [1]]), y=torch.ones(2))
    b = collate([d1, d2], lg_offset=mode)
    assert b.edge_index.tolist() == [[0, 1, 2, 0, 3, 4], [1, 2, 0, 2, 4, 3]]
    off = 3 if mode == "num_nodes" else 4  # PyG quirk: lg indices offset by the ATOM count
    assert b.lg_edge_index.tolist() == [[0, 1, off], [1, 2, off + 1]]
    assert b.batch.tolist() == [0, 0, 0, 1, 1] and b.ptr.tolist() == [0, 3, 5]
    assert b.y.shape == (4,)
