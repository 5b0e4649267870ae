"""Graph container and collation — the reference's PyG ``Data``/``Batch`` input contract.

The reference stores one ``torch_geometric.data.Data`` per material (``scripts/fetch.py:614-651``)
with attributes ``x, edge_index, edge_attr, lg_edge_index, lg_edge_attr, global_x, sg_one_hot, y``
and batches them with PyG's ``DataLoader`` (``scripts/train.py:2032-2044``).  PyG is not a
dependency of this engine, so this module provides the same duck type:

* ``Data`` — attribute bag, ``num_nodes == x.size(0)``, ``.to(device)``.
* ``Batch.from_data_list`` — PyG collation rules: tensors whose key contains
  ``index`` are concatenated along the last dim and offset by the cumulative ``num_nodes``
  (**including** ``lg_edge_index`` — PyG has no ``__inc__`` override for it), other
  tensors along dim 0; adds ``batch``, ``ptr``, ``num_graphs``.  ``lg_offset='num_edges'`` gives the
  corrected wiring for experiments; the default reproduces the reference bit for bit.
* ``DataLoader`` — ``torch.utils.data.DataLoader`` with that collate function.
"""
from __future__ import annotations

from typing import Any, Dict, List

import torch
import torch.utils.data


class Data:
    def __init__(self, **kwargs: Any) -> None:
        for k, v in kwargs.items():
            setattr(self, k, v)

    def keys(self) -> List[str]:
        return [k for k in self.__dict__.keys() if not k.startswith("_")]

    @property
    def num_nodes(self) -> int:
        return int(self.x.size(0))

    def to(self, device, non_blocking: bool = False) -> "Data":
        for k in self.keys():
            v = getattr(self, k)
            if isinstance(v, torch.Tensor):
                setattr(self, k, v.to(device, non_blocking=non_blocking))
        # device-side caches (CSR etc.) are per-device: drop them on a move
        self.__dict__.pop("_alignn_cache", None)
        return self

    def __repr__(self) -> str:
        parts = []
        for k in self.keys():
            v = getattr(self, k)
            parts.append(f"{k}={list(v.shape)}" if isinstance(v, torch.Tensor) else f"{k}=...")
        return f"{type(self).__name__}({', '.join(parts)})"


def _increment(key: str, d: Data, lg_offset: str) -> int:
    if "index" in key or key == "face":
        if key == "lg_edge_index" and lg_offset == "num_edges":
            return int(d.edge_index.size(1))
        return d.num_nodes
    return 0


class Batch(Data):
    @classmethod
    def from_data_list(cls, data_list: List[Data], lg_offset: str = "num_nodes") -> "Batch":
        if lg_offset not in ("num_nodes", "num_edges"):
            raise ValueError(f"lg_offset must be 'num_nodes' or 'num_edges', got {lg_offset!r}")
        if not data_list:
            raise ValueError("cannot collate an empty list")
        out = cls()
        for key in data_list[0].keys():
            vals = [getattr(d, key) for d in data_list]
            if not isinstance(vals[0], torch.Tensor):
                setattr(out, key, vals)
                continue
            cat_dim = -1 if ("index" in key or key == "face") else 0
            if vals[0].dim() == 0:
                vals = [v.view(1) for v in vals]
                cat_dim = 0
            cum, shifted = 0, []
            for d, v in zip(data_list, vals):
                shifted.append(v + cum if cum else v)
                cum += _increment(key, d, lg_offset)
            setattr(out, key, torch.cat(shifted, dim=cat_dim))
        counts = [d.num_nodes for d in data_list]
        out.batch = torch.repeat_interleave(torch.arange(len(counts)), torch.tensor(counts))
        out.ptr = torch.tensor([0] + torch.tensor(counts).cumsum(0).tolist(), dtype=torch.long)
        out.num_graphs = len(data_list)
        return out


class DataLoader(torch.utils.data.DataLoader):
    """``torch_geometric.loader.DataLoader`` look-alike (collates with :meth:`Batch.from_data_list`)."""

    def __init__(self, dataset, batch_size: int = 1, shuffle: bool = False, lg_offset: str = "num_nodes",
                 **kwargs: Any) -> None:
        kwargs.pop("collate_fn", None)
        self.lg_offset = lg_offset
        super().__init__(dataset, batch_size=batch_size, shuffle=shuffle,
                         collate_fn=lambda items: Batch.from_data_list(list(items), lg_offset=lg_offset),
                         **kwargs)


def batch_dims(batch: Data) -> Dict[str, int]:
    return {
        "num_nodes": int(batch.x.size(0)),
        "num_edges": int(batch.edge_index.size(1)),
        "num_triplets": int(batch.lg_edge_index.size(1)),
        "num_graphs": int(getattr(batch, "num_graphs", 1)),
    }
