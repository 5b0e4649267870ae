"""Shim ``torch_geometric.loader.DataLoader`` (PyG Collater over Batch.from_data_list)."""
from __future__ import annotations

import torch.utils.data

from .data import Batch


class DataLoader(torch.utils.data.DataLoader):
    def __init__(self, dataset, batch_size=1, shuffle=False, **kwargs):
        kwargs.pop("collate_fn", None)
        super().__init__(dataset, batch_size=batch_size, shuffle=shuffle,
                         collate_fn=lambda items: Batch.from_data_list(list(items)), **kwargs)
