"""ORACLE (test infrastructure only): restatement of the PyG 2.7.0 operators on the hot path.

The reference pins ``torch-geometric==2.7.0`` (``/root/reference/requirements.txt:9``) and calls:

* ``TransformerConv(D, D//H, heads=H, edge_dim=D, dropout=p, beta=True)``
  constructed at ``scripts/train.py:308`` and ``:326``, called at ``:315`` and ``:334``;
* ``global_mean_pool`` at ``scripts/train.py:388`` and ``:562``;
* ``DataLoader`` / ``Batch.from_data_list`` collation at ``scripts/train.py:2037``.

PyG is not installed here, so each function restates PyG's published algorithm (see SURVEY.md
§8a rows A5, A6, A9).  Functions are dtype-generic so fp64 ``gradcheck`` can be run on them.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F


# ----------------------------------------------------------------------------------------------
# torch_geometric.utils.scatter / softmax  ("exp(z - max_d z)/(sum + 1e-16)")
# ----------------------------------------------------------------------------------------------
def scatter_sum(src: torch.Tensor, index: torch.Tensor, dim_size: int) -> torch.Tensor:
    out = src.new_zeros((dim_size,) + tuple(src.shape[1:]))
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    return out.scatter_add_(0, idx, src)


def scatter_max(src: torch.Tensor, index: torch.Tensor, dim_size: int) -> torch.Tensor:
    # PyG: src.new_zeros(size).scatter_reduce_(0, index, src, 'amax', include_self=False);
    # empty segments therefore read 0 (they are never gathered back).
    out = src.new_zeros((dim_size,) + tuple(src.shape[1:]))
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    return out.scatter_reduce_(0, idx, src, reduce="amax", include_self=False)


def segment_softmax(src: torch.Tensor, index: torch.Tensor, num_nodes: int) -> torch.Tensor:
    """``torch_geometric.utils.softmax(src, index, num_nodes=N)`` (index path; ptr is None for a
    dense ``edge_index``).  The max is taken over the *detached* scores."""
    src_max = scatter_max(src.detach(), index, num_nodes)
    out = (src - src_max.index_select(0, index)).exp()
    out_sum = scatter_sum(out, index, num_nodes) + 1e-16
    return out / out_sum.index_select(0, index)


# ----------------------------------------------------------------------------------------------
# TransformerConv (concat=True, beta=True, root_weight=True, bias=True)
# ----------------------------------------------------------------------------------------------
def transformer_conv(
    x: torch.Tensor,
    edge_index: torch.Tensor,
    edge_attr: torch.Tensor,
    p: Dict[str, torch.Tensor],
    heads: int,
    dropout: float = 0.0,
    training: bool = False,
    return_alpha: bool = False,
):
    """Functional restatement of PyG 2.7.0 ``TransformerConv.forward``.

    ``p`` holds the module's parameters under their state-dict names
    (``lin_query.weight``, ``lin_key.bias``, ``lin_edge.weight``, ``lin_beta.weight``, ...).
    Flow is ``source_to_target``: j = edge_index[0] (source), i = edge_index[1] (target).
    """
    n = x.size(0)
    D_out = p["lin_query.weight"].size(0)
    H = heads
    C = D_out // H
    query = F.linear(x, p["lin_query.weight"], p["lin_query.bias"]).view(-1, H, C)
    key = F.linear(x, p["lin_key.weight"], p["lin_key.bias"]).view(-1, H, C)
    value = F.linear(x, p["lin_value.weight"], p["lin_value.bias"]).view(-1, H, C)
    src, dst = edge_index[0], edge_index[1]
    # MessagePassing.collect: x_i = x[index=edge_index[1]], x_j = x[edge_index[0]]
    query_i = query.index_select(0, dst)
    key_j = key.index_select(0, src)
    value_j = value.index_select(0, src)
    # message()
    e = F.linear(edge_attr, p["lin_edge.weight"]).view(-1, H, C)
    key_j = key_j + e
    alpha = (query_i * key_j).sum(dim=-1) / math.sqrt(C)
    alpha = segment_softmax(alpha, dst, n)
    alpha_saved = alpha
    alpha = F.dropout(alpha, p=dropout, training=training)
    msg = (value_j + e) * alpha.view(-1, H, 1)
    # aggregate (aggr='add')
    out = scatter_sum(msg, dst, n).view(-1, H * C)
    # root weight + beta gate
    x_r = F.linear(x, p["lin_skip.weight"], p["lin_skip.bias"])
    beta = F.linear(torch.cat([out, x_r, out - x_r], dim=-1), p["lin_beta.weight"]).sigmoid()
    out = beta * x_r + (1 - beta) * out
    if return_alpha:
        return out, alpha_saved
    return out


def global_mean_pool(x: torch.Tensor, batch: torch.Tensor, size: Optional[int] = None) -> torch.Tensor:
    """PyG ``global_mean_pool``: ``scatter(x, batch, reduce='mean')`` with size = batch.max()+1."""
    if size is None:
        size = int(batch.max().item()) + 1 if batch.numel() > 0 else 0
    total = scatter_sum(x, batch, size)
    count = scatter_sum(torch.ones_like(batch, dtype=x.dtype), batch, size).clamp(min=1)
    return total / count.view(-1, *([1] * (x.dim() - 1)))


# ----------------------------------------------------------------------------------------------
# Data / Batch.from_data_list (SURVEY §8a A9, §0.3 offset quirk)
# ----------------------------------------------------------------------------------------------
class RefData:
    """Minimal attribute bag with PyG ``Data`` semantics for num_nodes (= x.size(0))."""

    def __init__(self, **kw):
        for k, v in kw.items():
            setattr(self, k, v)

    def keys(self) -> List[str]:
        return [k for k in self.__dict__.keys()]

    @property
    def num_nodes(self) -> int:
        return int(self.x.size(0))


def _inc(key: str, data: RefData, lg_offset: str) -> int:
    # PyG Data.__inc__: 'batch' in key -> value.max()+1 ; 'index' in key or 'face' -> num_nodes ; else 0
    if "index" in key or key == "face":
        if key == "lg_edge_index" and lg_offset == "num_edges":
            return int(data.edge_index.size(1))
        return data.num_nodes
    return 0


def collate(data_list: List[RefData], lg_offset: str = "num_nodes") -> RefData:
    """Restatement of ``Batch.from_data_list``.  ``lg_offset='num_nodes'`` reproduces PyG exactly
    for the reference's ``Data`` (``lg_edge_index`` is a plain attribute, ``fetch.py:639``, no
    ``__inc__`` override).  ``'num_edges'`` is the corrected wiring, offered for comparison."""
    if lg_offset not in ("num_nodes", "num_edges"):
        raise ValueError(lg_offset)
    keys = data_list[0].keys()
    out = RefData()
    for key in keys:
        vals = [getattr(d, key) for d in data_list]
        if not isinstance(vals[0], torch.Tensor):
            setattr(out, key, vals)
            continue
        cat_dim = -1 if ("index" in key or key == "face") else 0
        if vals[0].dim() == 0:
            vals = [v.view(1) for v in vals]
            cat_dim = 0
        incs = []
        cum = 0
        for d in data_list:
            incs.append(cum)
            cum += _inc(key, d, lg_offset)
        if cum > 0:
            vals = [v + inc for v, inc in zip(vals, incs)]
        setattr(out, key, torch.cat(vals, dim=cat_dim))
    counts = [d.num_nodes for d in data_list]
    out.batch = torch.cat([torch.full((c,), i, dtype=torch.long) for i, c in enumerate(counts)])
    out.ptr = torch.tensor([0] + list(torch.tensor(counts).cumsum(0).tolist()), dtype=torch.long)
    out.num_graphs = len(data_list)
    return out
