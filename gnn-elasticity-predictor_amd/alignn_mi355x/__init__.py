"""alignn_mi355x — MI355X-native ALIGNN message-passing engine (drop-in for the hot path of
conorjmoran/gnn-elasticity-predictor ``scripts/train.py``).

Public API mirrors the reference: ``EdgeUpdateBlock``, ``NodeUpdateBlock``, ``AlignnRegressor``,
``HeteroAlignnRegressor``, ``TransformerConv`` (PyG parameter layout), ``Data``/``Batch``/
``DataLoader`` (PyG collation incl. the lg_edge_index offset rule), plus ``FusedTrainer`` (the
fused per-batch training step).  Compute runs in ``libalignn_hip.so`` (HIP, gfx950).
"""
from .data import Batch, Data, DataLoader  # noqa: F401
from .layout import AlignnConfig  # noqa: F401
from .model import (AlignnRegressor, EdgeUpdateBlock, HeteroAlignnRegressor, NodeUpdateBlock,  # noqa: F401
                    TransformerConv)
from .trainer import FusedTrainer  # noqa: F401

__version__ = "0.1.0"
