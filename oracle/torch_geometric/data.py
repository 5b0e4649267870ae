"""Shim ``torch_geometric.data``: Data / Batch / Dataset with PyG collation rules."""
from __future__ import annotations

import torch
from torch.utils.data import Dataset as _TorchDataset

from oracle.pyg_ref import RefData, collate


class Data(RefData):
    def to(self, device, non_blocking=False):
        for k, v in list(self.__dict__.items()):
            if isinstance(v, torch.Tensor):
                setattr(self, k, v.to(device))
        return self


class Batch(Data):
    @classmethod
    def from_data_list(cls, data_list, lg_offset="num_nodes"):
        b = collate(data_list, lg_offset=lg_offset)
        out = cls()
        out.__dict__.update(b.__dict__)
        return out


class Dataset(_TorchDataset):
    pass
