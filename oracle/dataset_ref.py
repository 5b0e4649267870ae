"""CPU restatement of the reference's dataset transform — TEST INFRASTRUCTURE ONLY (the product
path never imports oracle/).

Follows ``PtGraphDataset`` (``/root/reference/scripts/train.py:49-216``): ``_is_valid`` (:174-182),
the node-dimension rules (:95-117), ``__getitem__``'s select / pad / truncate and reshapes
(:137-169) and ``_apply_standardization`` (:200-216); and the train-only feature statistics of
``_setup`` (:1324-1380).  Pinned by ``tests/golden/dataset.npz``, which the reference's own classes
wrote (``tests/golden/make_golden_dataset.py``).
"""
from __future__ import annotations

from typing import Dict, List, Optional

import torch

FIELDS = ("x", "edge_attr", "lg_edge_attr", "global_x", "sg_one_hot", "y")


def is_valid(g: Dict[str, torch.Tensor]) -> bool:
    """train.py:174-182."""
    for k in FIELDS:
        t = g.get(k)
        if t is not None and (torch.isnan(t).any() or torch.isinf(t).any()):
            return False
    return True


def node_dims(raw_node_dim: int, use_mat2vec: bool = True, force_node_dim: Optional[int] = None):
    """(scalar_dim, mat2vec_dim, node_dim, use_mat2vec) as train.py:102-117."""
    scalar = min(6, raw_node_dim)
    raw_m2v = max(0, raw_node_dim - scalar)
    m2v = raw_m2v if use_mat2vec else 0
    if force_node_dim is not None:
        if force_node_dim < scalar:
            raise ValueError("forced node dimension below the scalar dimension")
        m2v = max(force_node_dim - scalar, 0)
        use_mat2vec = m2v > 0
    return scalar, m2v, scalar + m2v, use_mat2vec


def item(g: Dict[str, torch.Tensor], raw_node_dim: int, use_mat2vec: bool = True,
         force_node_dim: Optional[int] = None, stats: Optional[Dict[str, Optional[torch.Tensor]]] = None):
    """(x, global_x) of PtGraphDataset.__getitem__ (train.py:137-172) for one stored graph."""
    scalar, m2v, node_dim, use_m2v = node_dims(raw_node_dim, use_mat2vec, force_node_dim)
    x = g["x"].reshape(-1, raw_node_dim).clone()
    if not use_m2v and raw_node_dim - scalar > 0:
        x = x[:, :scalar]
    if x.size(1) < node_dim:
        x = torch.cat([x, torch.zeros(x.size(0), node_dim - x.size(1), dtype=x.dtype)], 1)
    elif x.size(1) > node_dim:
        x = x[:, :node_dim]
    gx = g["global_x"].reshape(-1, 1).clone()
    st = stats or {}
    if scalar > 0 and st.get("scalar_mean") is not None and st.get("scalar_std") is not None:
        x[:, :scalar] = (x[:, :scalar] - st["scalar_mean"]) / st["scalar_std"]
    if m2v > 0 and st.get("embed_mean") is not None and st.get("embed_std") is not None:
        x[:, scalar:] = (x[:, scalar:] - st["embed_mean"]) / st["embed_std"]
    if gx.numel() > 0 and st.get("global_mean") is not None and st.get("global_std") is not None:
        gx = ((gx.reshape(-1) - st["global_mean"]) / st["global_std"]).reshape(gx.shape)
    return x, gx


def feature_stats(graphs: List[Dict[str, torch.Tensor]], train_idx, raw_node_dim: int, use_mat2vec: bool = True,
                  force_node_dim: Optional[int] = None, eps: float = 1e-12) -> Dict[str, Optional[torch.Tensor]]:
    """train.py:1324-1380 over the (unstandardized) items of ``graphs[train_idx]``."""
    scalar, m2v, _, _ = node_dims(raw_node_dim, use_mat2vec, force_node_dim)
    gdim = graphs[0]["global_x"].numel()
    tot = 0
    ss, sq = torch.zeros(scalar, dtype=torch.double), torch.zeros(scalar, dtype=torch.double)
    es, eq = torch.zeros(m2v, dtype=torch.double), torch.zeros(m2v, dtype=torch.double)
    gs, gq = torch.zeros(gdim, dtype=torch.double), torch.zeros(gdim, dtype=torch.double)
    for i in train_idx:
        x, gx = item(graphs[i], raw_node_dim, use_mat2vec, force_node_dim)
        x = x.double()
        tot += x.size(0)
        ss += x[:, :scalar].sum(0)
        sq += (x[:, :scalar] ** 2).sum(0)
        if m2v:
            es += x[:, scalar:].sum(0)
            eq += (x[:, scalar:] ** 2).sum(0)
        g = gx.double().reshape(-1)
        gs += g
        gq += g ** 2
    out: Dict[str, Optional[torch.Tensor]] = {}

    def ms(s, q, n):
        mean = s / n
        var = torch.clamp(q / n - mean ** 2, min=eps)
        return mean.float(), torch.sqrt(var).float()

    out["scalar_mean"], out["scalar_std"] = ms(ss, sq, tot)
    out["embed_mean"], out["embed_std"] = ms(es, eq, tot) if m2v else (None, None)
    out["global_mean"], out["global_std"] = ms(gs, gq, len(train_idx))
    return out
