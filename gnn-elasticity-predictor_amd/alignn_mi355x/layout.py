"""Flat parameter layout of the ALIGNN regressor.

Every trainable tensor of ``HeteroAlignnRegressor`` (state-dict names of the reference,
SURVEY §8b) lives in ONE contiguous fp32 buffer, ordered so that the engine's fused operands are
plain views (no per-step concatenation):

* per TransformerConv: ``[W_query; W_key; W_value; W_skip]`` as one [4D, D] matrix and the four
  biases as one [4D] vector (the engine's QKVR projection is a single GEMM);
* ``logvar_heads`` last, so the reference's two optimizer groups (train.py:1516-1531: base +
  mean heads, and logvar heads) are two contiguous segments.

``base.output_heads`` are registered (checkpoint compatibility) but unused by the hetero forward
(train.py:579-586), so they stay outside the buffer and never receive gradients.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Tuple


@dataclass(frozen=True)
class AlignnConfig:
    node_dim: int
    edge_dim: int
    angle_dim: int
    global_dim: int
    target_dim: int
    hidden: int = 256
    layers: int = 4
    heads: int = 4
    dropout: float = 0.15

    def validate(self) -> None:
        if self.heads <= 0:
            raise ValueError("heads must be positive")
        if self.target_dim <= 0:
            raise ValueError("target_dim must be positive")
        if self.hidden % self.heads != 0:
            raise ValueError("hidden size must be divisible by number of heads")


def _linear(prefix: str, fin: int, fout: int, bias: bool = True) -> List[Tuple[str, Tuple[int, ...]]]:
    out = [(prefix + "weight", (fout, fin))]
    if bias:
        out.append((prefix + "bias", (fout,)))
    return out


def conv_entries(prefix: str, D: int, H: int, edge_dim: int) -> List[Tuple[str, Tuple[int, ...]]]:
    """A TransformerConv's parameters except lin_edge (kept with the tail group, flat_entries)."""
    HC = D  # heads * out_channels with out_channels = D // H
    c = prefix + "conv."
    return [
        (c + "lin_query.weight", (HC, D)),
        (c + "lin_key.weight", (HC, D)),
        (c + "lin_value.weight", (HC, D)),
        (c + "lin_skip.weight", (HC, D)),
        (c + "lin_query.bias", (HC,)),
        (c + "lin_key.bias", (HC,)),
        (c + "lin_value.bias", (HC,)),
        (c + "lin_skip.bias", (HC,)),
        (c + "lin_beta.weight", (1, 3 * HC)),
    ]


def flat_entries(cfg: AlignnConfig, hetero: bool = True) -> List[Tuple[str, Tuple[int, ...]]]:
    """``hetero``: HeteroAlignnRegressor (mean/logvar heads; output_heads excluded) or the base
    AlignnRegressor (output_heads, train.py:373/:400).

    Order = the order in which the backward completes the gradients (two data-parallel buckets,
    dp.GradBuckets): first every conv block's own projections, gate and LayerNorm (written by the
    per-layer backward, engine._backward_layers), then what the backward's tail writes — the encoders,
    the edge projections folded into the convs (lin_edge, edge_proj: their chain rules run after the
    layers), the readout and the heads (logvar heads last: the second optimizer group)."""
    D = cfg.hidden
    e: List[Tuple[str, Tuple[int, ...]]] = []
    for l in range(cfg.layers):
        p = f"base.edge_blocks.{l}."
        e += conv_entries(p, D, cfg.heads, D)
        e += [(p + "norm.weight", (D,)), (p + "norm.bias", (D,))]
    for l in range(cfg.layers):
        p = f"base.node_blocks.{l}."
        e += conv_entries(p, D, cfg.heads, D)
        e += [(p + "norm.weight", (D,)), (p + "norm.bias", (D,))]
    e += _linear("base.node_encoder.0.", cfg.node_dim, D) + _linear("base.node_encoder.2.", D, D)
    e += _linear("base.edge_encoder.0.", cfg.edge_dim, D) + _linear("base.edge_encoder.2.", D, D)
    if cfg.angle_dim > 0:
        e += _linear("base.angle_encoder.0.", cfg.angle_dim, D) + _linear("base.angle_encoder.2.", D, D)
    # per-layer blocks at a constant stride (FlatViews._stack)
    e += [(f"base.edge_blocks.{l}.conv.lin_edge.weight", (D, D)) for l in range(cfg.layers)]
    e += [(f"base.node_blocks.{l}.conv.lin_edge.weight", (D, D)) for l in range(cfg.layers)]
    e += [(f"base.node_blocks.{l}.edge_proj.weight", (D, D)) for l in range(cfg.layers)]
    e += [(f"base.node_blocks.{l}.edge_proj.bias", (D,)) for l in range(cfg.layers)]
    e += _linear("base.feat_proj.0.", D + cfg.global_dim, D)
    if not hetero:
        e = [(k[len("base."):], s) for k, s in e]
        for t in range(cfg.target_dim):
            e += [(f"output_heads.{t}.weight", (1, D))]
        for t in range(cfg.target_dim):
            e += [(f"output_heads.{t}.bias", (1,))]
        return e
    for t in range(cfg.target_dim):
        e += [(f"mean_heads.{t}.weight", (1, D))]
    for t in range(cfg.target_dim):
        e += [(f"mean_heads.{t}.bias", (1,))]
    for t in range(cfg.target_dim):
        e += [(f"logvar_heads.{t}.weight", (1, D))]
    for t in range(cfg.target_dim):
        e += [(f"logvar_heads.{t}.bias", (1,))]
    return e


def bucket_split(cfg: AlignnConfig, hetero: bool = True) -> int:
    """Flat offset where the tail group starts: [0, split) holds the conv blocks' own parameters,
    whose gradients are final once the per-layer backward is done (dp.GradBuckets)."""
    offs, total, _ = offsets(cfg, hetero)
    return offs[("base." if hetero else "") + "node_encoder.0.weight"][0]


def offsets(cfg: AlignnConfig, hetero: bool = True) -> Tuple[Dict[str, Tuple[int, Tuple[int, ...]]], int, int]:
    """name -> (offset, shape); total size; offset where the logvar-head segment starts."""
    out: Dict[str, Tuple[int, Tuple[int, ...]]] = {}
    pos = 0
    sigma_start = None
    for name, shape in flat_entries(cfg, hetero):
        if sigma_start is None and name.startswith("logvar_heads."):
            sigma_start = pos
        n = 1
        for s in shape:
            n *= s
        out[name] = (pos, shape)
        pos += n
    return out, pos, sigma_start if sigma_start is not None else pos
