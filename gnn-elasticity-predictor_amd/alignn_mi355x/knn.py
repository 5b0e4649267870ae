"""KNN density weighting of training samples.

Reference: ``compute_global_knn_weights`` (scripts/train.py:930-1010) — embed every training graph
with ``model.embed``, standardize, find each sample's k nearest neighbours (sklearn, host), weight by
inverse local density and local label noise, clip, normalise; the weights then scale the per-graph
NLL (train.py:660-674; here ``FusedTrainer.step(batch, sample_weights=...)``).

MI355X: embeddings by the engine (eval mode), standardisation by HIP kernels + the two-stage column
sums, the Gram matrix by the MFMA GEMM (row blocks, so n^2 never has to fit at once), and the
neighbour selection + weight formula by one wave per query row (``alignn_knn_select_weights``).
Clip and mean-normalisation run on the host over the n weights, as in the reference.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import _lib, infer, ops
from .engine import batch_cache
from .ops import stream_ptr


def embed_collect(model, batches) -> Tuple[torch.Tensor, torch.Tensor, np.ndarray]:
    """(Z [n, D], Y [n, T] raw targets, train_idx [n]) over the batches, Z/Y on the device."""
    zs, ys, idx = [], [], []
    for b in batches:
        zs.append(infer.forward(model, b, "embed").clone())   # a replayed plan once the signature repeats
        ys.append(b.y.view(b.num_graphs, -1).float())
        if not hasattr(b, "train_idx"):
            raise ValueError("KNN weighting requires 'train_idx' on each batch.")
        idx.append(b.train_idx.view(-1).cpu().numpy())
    if not zs:
        raise ValueError("No batches produced embeddings for KNN weighting.")
    return torch.cat(zs).contiguous(), torch.cat(ys).contiguous(), np.concatenate(idx)


def knn_raw_weights(Z: torch.Tensor, Y: torch.Tensor, k: int, eps: float, alpha: float, beta: float,
                    block_rows: int = 8192) -> torch.Tensor:
    """Device [n] weights before clip / normalisation."""
    n, D = Z.shape
    T = Y.size(1)
    k_eff = max(1, min(int(k), n - 1))
    lib = _lib.lib()
    s = stream_ptr()
    colsum = torch.empty(D, device=Z.device)
    ops.colsum(Z, colsum)
    sq = torch.empty_like(Z)
    _lib.check(lib.alignn_col_center_sq_f32(Z.data_ptr(), n, D, colsum.data_ptr(), sq.data_ptr(), s),
               "alignn_col_center_sq_f32")
    ssq = torch.empty(D, device=Z.device)
    ops.colsum(sq, ssq)
    Zs = torch.empty_like(Z)
    _lib.check(lib.alignn_standardize_f32(Z.data_ptr(), n, D, colsum.data_ptr(), ssq.data_ptr(), Zs.data_ptr(), s),
               "alignn_standardize_f32")
    r = torch.empty(n, device=Z.device)
    _lib.check(lib.alignn_row_sqnorm_f32(Zs.data_ptr(), n, D, r.data_ptr(), s), "alignn_row_sqnorm_f32")
    w = torch.empty(n, device=Z.device)
    rows = min(n, block_rows)
    G = torch.empty(rows, n, device=Z.device)
    for r0 in range(0, n, rows):
        m = min(rows, n - r0)
        ops.gemm(Zs[r0:r0 + m], Zs.t(), G[:m])
        _lib.check(lib.alignn_knn_select_weights(G.data_ptr(), G.stride(0), r.data_ptr(), n, r0, m, k_eff,
                                                 Y.data_ptr(), T, float(eps), float(alpha), float(beta), None,
                                                 w.data_ptr(), s), "alignn_knn_select_weights")
    return w


def compute_global_knn_weights(model, batches, *, k: int = 20, eps: float = 1e-6, alpha: float = 0.75,
                               beta: float = 1.0, clip_min: Optional[float] = 0.2,
                               clip_max: Optional[float] = 1.0) -> Dict[int, float]:
    """train.py:930-1010: {train_idx: weight}; defaults are the reference's CLI defaults (:1184-1189)."""
    Z, Y, idx = embed_collect(model, batches)
    w = knn_raw_weights(Z, Y, k, eps, alpha, beta).double().cpu()
    if clip_min is not None:
        w = torch.clamp(w, min=float(clip_min))
    if clip_max is not None:
        w = torch.clamp(w, max=float(clip_max))
    w = w / (w.mean() + 1e-12)
    return {int(i): float(x) for i, x in zip(idx.tolist(), w.tolist())}


def batch_weights(weight_map: Dict[int, float], batch, device) -> torch.Tensor:
    """Per-graph weights of a batch from its train_idx (train.py:661-674, same error on gaps)."""
    ids = batch.train_idx.view(-1).cpu().tolist()
    missing = [int(i) for i in ids if int(i) not in weight_map]
    if missing:
        raise RuntimeError(f"KNN weight map missing {len(missing)}/{len(ids)} train_idx ids; examples: {missing[:5]}")
    return torch.tensor([float(weight_map[int(i)]) for i in ids], dtype=torch.float32, device=device)
