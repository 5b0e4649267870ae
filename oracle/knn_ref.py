"""ORACLE — test infrastructure only (never imported by the product path).

CPU restatement of ``compute_global_knn_weights`` (scripts/train.py:930-1010) from the embeddings
on: standardize, k nearest neighbours by euclidean distance (exact, float64 brute force instead of
sklearn's NearestNeighbors), density rho = k / (sum of the k distances + eps), w = rho^-alpha,
w /= 1 + beta * mean_t var_k(y of the neighbours), clip, w /= mean(w) + 1e-12.  Pinned by
tests/golden/knn.npz, which the reference's own function wrote (tests/golden/make_golden_knn.py).
"""
from __future__ import annotations

from typing import Optional

import torch


def knn_weights(Z: torch.Tensor, Y: torch.Tensor, k: int, eps: float, alpha: float, beta: float,
                clip_min: Optional[float], clip_max: Optional[float]) -> torch.Tensor:
    Z = Z.double()
    Y = Y.double()
    Zs = (Z - Z.mean(0)) / Z.std(0, unbiased=False).clamp_min(1e-8)
    n = Zs.size(0)
    k_eff = max(1, min(int(k), n - 1))
    D = torch.cdist(Zs, Zs)
    D.fill_diagonal_(float("inf"))
    d, ind = torch.topk(D, k_eff, dim=1, largest=False)
    rho = k_eff / (d.sum(1) + eps)
    w = rho.pow(-alpha)
    w = w / (1.0 + beta * Y[ind].var(dim=1, unbiased=False).mean(dim=1))
    if clip_min is not None:
        w = w.clamp(min=clip_min)
    if clip_max is not None:
        w = w.clamp(max=clip_max)
    return w / (w.mean() + 1e-12)
