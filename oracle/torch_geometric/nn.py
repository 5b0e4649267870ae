"""Shim ``torch_geometric.nn``: TransformerConv module + global_mean_pool over oracle.pyg_ref."""
from __future__ import annotations

import torch
from torch import nn

from oracle.pyg_ref import global_mean_pool, transformer_conv  # noqa: F401


class TransformerConv(nn.Module):
    """Parameter layout of PyG 2.7.0 ``TransformerConv`` (registration order lin_key, lin_query,
    lin_value, lin_edge, lin_skip, lin_beta) with concat=True, root_weight=True, bias=True."""

    def __init__(self, in_channels, out_channels, heads=1, concat=True, beta=False, dropout=0.0,
                 edge_dim=None, bias=True, root_weight=True, **kwargs):
        super().__init__()
        assert concat and root_weight and bias and beta and edge_dim is not None
        self.in_channels, self.out_channels, self.heads = in_channels, out_channels, heads
        self.beta, self.dropout, self.edge_dim = beta, dropout, edge_dim
        HC = heads * out_channels
        self.lin_key = nn.Linear(in_channels, HC)
        self.lin_query = nn.Linear(in_channels, HC)
        self.lin_value = nn.Linear(in_channels, HC)
        self.lin_edge = nn.Linear(edge_dim, HC, bias=False)
        self.lin_skip = nn.Linear(in_channels, HC, bias=bias)
        self.lin_beta = nn.Linear(3 * HC, 1, bias=False)

    def forward(self, x, edge_index, edge_attr=None):
        p = {k: v for k, v in self.state_dict(keep_vars=True).items()}
        return transformer_conv(x, edge_index, edge_attr, p, self.heads, dropout=self.dropout,
                                training=self.training)
