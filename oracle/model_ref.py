"""ORACLE (test infrastructure only): PyTorch-CPU restatement of the reference model and step.

Follows ``/root/reference/scripts/train.py``:

* ``EdgeUpdateBlock.forward``      train.py:312-317
* ``NodeUpdateBlock.forward``      train.py:330-336
* encoders                          train.py:350-364 (used at :547-556)
* ``HeteroAlignnRegressor._shared`` train.py:537-574, ``forward`` :579-586
* hetero NLL loss                   train.py:655-681
* clip + AdamW step                 train.py:697-699, optimizer :1516-1542

The model is a pure function of a state dict (keys identical to the reference's),
so the same fixture drives the oracle, the reference-through-shim and the HIP engine.
"""
from __future__ import annotations

import math
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from .pyg_ref import global_mean_pool, transformer_conv

MIN_LOGVAR_FLOOR = -2.9  # train.py:39


def _sub(state: Dict[str, torch.Tensor], prefix: str) -> Dict[str, torch.Tensor]:
    n = len(prefix)
    return {k[n:]: v for k, v in state.items() if k.startswith(prefix)}


def _mlp2(x, st, prefix):
    # nn.Sequential(Linear, ReLU, Linear)  (train.py:350-364)
    h = F.relu(F.linear(x, st[prefix + "0.weight"], st[prefix + "0.bias"]))
    return F.linear(h, st[prefix + "2.weight"], st[prefix + "2.bias"])


def edge_block(st, prefix, edge_state, lg_edge_index, angle_emb, heads, dropout=0.0, training=False):
    """train.py:312-317"""
    if edge_state.numel() == 0 or angle_emb.numel() == 0 or lg_edge_index.numel() == 0:
        return edge_state
    out = transformer_conv(edge_state, lg_edge_index, angle_emb, _sub(st, prefix + "conv."), heads,
                           dropout=dropout, training=training)
    out = F.layer_norm(out, (out.size(-1),), st[prefix + "norm.weight"], st[prefix + "norm.bias"], 1e-5)
    return edge_state + F.dropout(F.relu(out), p=dropout, training=training)


def node_block(st, prefix, node_state, edge_index, edge_state, heads, dropout=0.0, training=False):
    """train.py:330-336"""
    if edge_state.numel() == 0 or edge_index.numel() == 0:
        return node_state
    edge_attr = F.linear(edge_state, st[prefix + "edge_proj.weight"], st[prefix + "edge_proj.bias"])
    out = transformer_conv(node_state, edge_index, edge_attr, _sub(st, prefix + "conv."), heads,
                           dropout=dropout, training=training)
    out = F.layer_norm(out, (out.size(-1),), st[prefix + "norm.weight"], st[prefix + "norm.bias"], 1e-5)
    return node_state + F.dropout(F.relu(out), p=dropout, training=training)


def num_layers(st: Dict[str, torch.Tensor]) -> int:
    l = 0
    while f"base.edge_blocks.{l}.norm.weight" in st:
        l += 1
    return l


def hetero_forward(st, data, heads, dropout=0.0, training=False, return_shared=False, retain=None):
    """``HeteroAlignnRegressor.forward`` (train.py:537-586).  Returns (mean [B,T], logvar [B,T])."""
    hidden = st["base.node_encoder.2.weight"].size(0)
    node_state = _mlp2(data.x, st, "base.node_encoder.")
    if data.edge_attr.numel() > 0:
        edge_state = _mlp2(data.edge_attr, st, "base.edge_encoder.")
    else:
        edge_state = torch.zeros(data.edge_index.size(1), node_state.size(-1), dtype=node_state.dtype)
    has_angle = "base.angle_encoder.0.weight" in st
    if has_angle and data.lg_edge_attr.numel() > 0:
        angle_emb = _mlp2(data.lg_edge_attr, st, "base.angle_encoder.")
    else:
        angle_emb = torch.zeros(data.lg_edge_index.size(1), edge_state.size(-1), dtype=node_state.dtype)
    if retain is not None:
        edge_state.retain_grad()
        retain["e0"] = edge_state
    for l in range(num_layers(st)):
        edge_state = edge_block(st, f"base.edge_blocks.{l}.", edge_state, data.lg_edge_index, angle_emb,
                                heads, dropout, training)
        if retain is not None:
            edge_state.retain_grad()
            retain[f"e{l + 1}"] = edge_state
        node_state = node_block(st, f"base.node_blocks.{l}.", node_state, data.edge_index, edge_state,
                                heads, dropout, training)
        if retain is not None:
            node_state.retain_grad()
            retain[f"h{l + 1}"] = node_state
    pooled = global_mean_pool(node_state, data.batch)
    global_x = data.global_x
    if global_x.dim() == 1:
        global_x = global_x.unsqueeze(0)
    global_x = global_x.reshape(pooled.size(0), -1)
    sg = data.sg_one_hot
    if sg.dim() == 1:
        sg = sg.unsqueeze(0)
    sg = sg.reshape(pooled.size(0), -1)
    feats = torch.cat([pooled, torch.cat([global_x, sg], dim=1)], dim=1)
    feats = F.dropout(feats, p=dropout, training=training)
    shared = F.relu(F.linear(feats, st["base.feat_proj.0.weight"], st["base.feat_proj.0.bias"]))
    shared = F.dropout(shared, p=dropout, training=training)
    if return_shared:
        return shared
    t = 0
    means, logvars = [], []
    while f"mean_heads.{t}.weight" in st:
        means.append(F.linear(shared, st[f"mean_heads.{t}.weight"], st[f"mean_heads.{t}.bias"]))
        logvars.append(F.linear(shared, st[f"logvar_heads.{t}.weight"], st[f"logvar_heads.{t}.bias"]))
        t += 1
    return torch.cat(means, dim=1), torch.cat(logvars, dim=1)


def log_transform(y: torch.Tensor, means, stds) -> torch.Tensor:
    """``LogTransformer.transform_tensor`` (train.py:268-280)."""
    m = torch.as_tensor(means, dtype=y.dtype).view(1, -1)
    s = torch.as_tensor(stds, dtype=y.dtype).view(1, -1)
    return (torch.log(y) - m) / s


def hetero_loss(mean, logvar, target_trans, log_sigma_l2=0.1, floor=MIN_LOGVAR_FLOOR):
    """Loss of ``train_epoch_hetero`` (train.py:656-681), no KNN sample weights."""
    logvar = torch.clamp(logvar, min=floor)
    var = torch.exp(logvar)
    diff = mean - target_trans.to(mean.dtype)
    nll = 0.5 * (logvar + diff.pow(2) / var)
    sample_loss = nll.mean(dim=1)
    loss = sample_loss.mean()
    if log_sigma_l2 > 0.0:
        loss = loss + float(log_sigma_l2) * (0.5 * logvar).pow(2).mean()
    return loss


def param_order(st: Dict[str, torch.Tensor]):
    """Parameter order of ``HeteroAlignnRegressor.parameters()`` (registration order)."""
    return list(st.keys())


def train_step(st: Dict[str, torch.Tensor], data, heads, target_means, target_stds,
               lr=3e-4, weight_decay=1e-4, log_sigma_l2=0.1, max_norm=5.0, steps=1,
               opt_state=None):
    """One reference training step (train.py:647-699) at dropout 0 and jitter 0, CPU fp32 path:
    forward -> hetero NLL -> backward -> clip_grad_norm_(5) -> AdamW (two groups, same lr).
    Returns (loss, grads_before_clip, new_state)."""
    params = {k: v.detach().clone().requires_grad_(True) for k, v in st.items()}
    base = [params[k] for k in params if not k.startswith("logvar_heads.")]
    sigma = [params[k] for k in params if k.startswith("logvar_heads.")]
    opt = torch.optim.AdamW([{"params": base, "lr": lr}, {"params": sigma, "lr": lr}], lr=lr,
                            weight_decay=weight_decay)
    losses, grads = [], None
    for _ in range(steps):
        opt.zero_grad(set_to_none=True)
        target = data.y.view(data.num_graphs, -1)
        tt = log_transform(target, target_means, target_stds)
        mean, logvar = hetero_forward(params, data, heads)
        loss = hetero_loss(mean, logvar, tt, log_sigma_l2)
        loss.backward()
        grads = {k: v.grad.detach().clone() for k, v in params.items() if v.grad is not None}
        torch.nn.utils.clip_grad_norm_(list(params.values()), max_norm=max_norm)
        opt.step()
        losses.append(float(loss.detach()))
    return losses, grads, {k: v.detach().clone() for k, v in params.items()}
