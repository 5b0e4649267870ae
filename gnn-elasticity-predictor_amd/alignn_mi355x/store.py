"""Dataset resident in HBM + on-device batch assembly.

The reference keeps one ``torch.save``d PyG ``Data`` per material and pays a ``torch.load`` per
sample per step (``scripts/train.py:132``), then collates on the host (PyG ``Collater``, SURVEY §8a
A9).  On MI355X the whole dataset fits in HBM many times over (10k MP-like graphs ≈ 5 GB fp32 of
288 GB), so :class:`GraphStore` uploads every field once as one flat array with per-graph row
ranges, and :meth:`GraphStore.collate` builds a batch with three HIP kernels (segmented row copies,
two-row index copies with PyG's increments, the ``batch`` vector).  The host work per batch is a
few prefix sums over the selected graphs and one small upload.

Collation rules are PyG's (identical to :meth:`alignn_mi355x.data.Batch.from_data_list`): tensors
with ``index`` in the key are concatenated along the last dim and shifted by the cumulative
``num_nodes`` — including ``lg_edge_index`` (``lg_offset='num_nodes'``, the reference's behaviour,
SURVEY §0.3); ``lg_offset='num_edges'`` gives the corrected wiring.  Other tensors are concatenated
along dim 0.

On disk: a directory of ``<field>.npy`` arrays plus ``meta.json`` (no pickles; loaded with
``numpy.load(mmap_mode='r')``), written by :meth:`GraphStore.save`.
"""
from __future__ import annotations

import json
import os
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch

from . import _lib
from .data import Batch, Data
from .ops import stream_ptr


def _excl_cumsum(a: np.ndarray) -> np.ndarray:
    out = np.zeros(len(a), dtype=np.int64)
    if len(a) > 1:
        np.cumsum(a[:-1], out=out[1:])
    return out


class CollatePlan:
    """Host part of a collate: per field and selected graph, source start, destination start,
    row count, and (index fields) the increment.  Pure numpy (tested on CPU against PyG's rules)."""

    def __init__(self, store_meta: Dict, counts: Dict[str, np.ndarray], starts: Dict[str, np.ndarray],
                 idx: np.ndarray, lg_offset: str):
        if lg_offset not in ("num_nodes", "num_edges"):
            raise ValueError(f"lg_offset must be 'num_nodes' or 'num_edges', got {lg_offset!r}")
        self.idx = idx
        self.fields = {}
        nodes = counts["x"][idx]
        node_inc = _excl_cumsum(nodes)
        for f, m in store_meta.items():
            cnt = counts[f][idx].astype(np.int64)
            ent = {"src": starts[f][idx].astype(np.int64), "dst": _excl_cumsum(cnt), "count": cnt,
                   "total": int(cnt.sum()), "max": int(cnt.max()) if len(cnt) else 0}
            if m["kind"] == "index":
                if f == "lg_edge_index" and lg_offset == "num_edges":
                    ent["add"] = _excl_cumsum(counts["edge_index"][idx].astype(np.int64))
                else:
                    ent["add"] = node_inc
            self.fields[f] = ent
        self.nodes = nodes.astype(np.int64)
        self.node_dst = node_inc
        self.ptr = np.concatenate([[0], np.cumsum(self.nodes)]).astype(np.int64)

    def apply_host(self, host_arrays: Dict[str, np.ndarray], store_meta: Dict) -> Dict[str, np.ndarray]:
        """Numpy emulation of the device kernels (test reference for the plan)."""
        out = {}
        for f, ent in self.fields.items():
            a = host_arrays[f]
            if store_meta[f]["kind"] == "index":
                parts = [a[:, s:s + c] + add for s, c, add in zip(ent["src"], ent["count"], ent["add"])]
                out[f] = np.concatenate(parts, axis=1) if parts else a[:, :0]
            else:
                parts = [a[s:s + c] for s, c in zip(ent["src"], ent["count"])]
                out[f] = np.concatenate(parts, axis=0)
        out["batch"] = np.repeat(np.arange(len(self.nodes), dtype=np.int64), self.nodes)
        out["ptr"] = self.ptr
        return out


class GraphStore:
    def __init__(self, arrays: Dict[str, torch.Tensor], counts: Dict[str, np.ndarray], meta: Dict,
                 extras: Optional[Dict[str, List]] = None):
        self.arrays = arrays          # field -> device tensor ([total, width] float32 or [2, total] int64)
        self.counts = counts          # field -> int64 [num_graphs] rows per graph
        self.meta = meta              # field -> {"kind": "rows"|"index", "shape": trailing shape}
        self.starts = {f: _excl_cumsum(c) for f, c in counts.items()}
        self.extras = extras or {}    # non-tensor per-graph attributes (e.g. material ids)
        self.num_graphs = len(next(iter(counts.values())))
        self._staging = None

    # -------------------------------------------------------------------------------- building
    @classmethod
    def host_arrays(cls, data_list: Sequence[Data]):
        """(arrays, counts, meta, extras) in host numpy form from a list of Data."""
        if not data_list:
            raise ValueError("empty dataset")
        first = data_list[0]
        arrays, counts, meta, extras = {}, {}, {}, {}
        for key in first.keys():
            v0 = getattr(first, key)
            if not isinstance(v0, torch.Tensor):
                extras[key] = [getattr(d, key) for d in data_list]
                continue
            vals = [getattr(d, key) for d in data_list]
            if "index" in key:
                if v0.dim() != 2 or v0.size(0) != 2:
                    raise ValueError(f"{key}: index fields must be [2, m]")
                arrays[key] = np.concatenate([v.to(torch.int64).numpy() for v in vals], axis=1)
                counts[key] = np.asarray([v.size(1) for v in vals], dtype=np.int64)
                meta[key] = {"kind": "index", "shape": []}
            else:
                vals = [v.reshape(1) if v.dim() == 0 else v for v in vals]
                shape = list(vals[0].shape[1:])
                width = int(np.prod(shape)) if shape else 1
                arrays[key] = np.concatenate([v.to(torch.float32).reshape(v.size(0), width).numpy() for v in vals], 0)
                counts[key] = np.asarray([v.size(0) for v in vals], dtype=np.int64)
                meta[key] = {"kind": "rows", "shape": shape, "width": width}
        if "x" not in arrays:
            raise ValueError("graphs need node features 'x'")
        return arrays, counts, meta, extras

    @classmethod
    def from_data_list(cls, data_list: Sequence[Data], device) -> "GraphStore":
        arrays, counts, meta, extras = cls.host_arrays(data_list)
        dev = {k: torch.from_numpy(np.ascontiguousarray(v)).to(device) for k, v in arrays.items()}
        return cls(dev, counts, meta, extras)

    def save(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        for k, v in self.arrays.items():
            np.save(os.path.join(path, f"{k}.npy"), v.cpu().numpy())
            np.save(os.path.join(path, f"{k}.counts.npy"), self.counts[k])
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump({"fields": self.meta, "extras": {k: [str(x) for x in v] for k, v in self.extras.items()}}, f)

    @classmethod
    def load(cls, path: str, device) -> "GraphStore":
        with open(os.path.join(path, "meta.json")) as f:
            m = json.load(f)
        arrays, counts = {}, {}
        for k in m["fields"]:
            a = np.load(os.path.join(path, f"{k}.npy"), mmap_mode="r")      # no pickles
            arrays[k] = torch.from_numpy(np.ascontiguousarray(a)).to(device)
            counts[k] = np.load(os.path.join(path, f"{k}.counts.npy"))
        return cls(arrays, counts, m["fields"], m.get("extras", {}))

    # -------------------------------------------------------------------------------- batches
    def plan(self, indices, lg_offset: str = "num_nodes") -> CollatePlan:
        idx = np.asarray(indices, dtype=np.int64).reshape(-1)
        if idx.size == 0:
            raise ValueError("cannot collate an empty list")
        if idx.min() < 0 or idx.max() >= self.num_graphs:
            raise IndexError("graph index out of range")
        return CollatePlan(self.meta, self.counts, self.starts, idx, lg_offset)

    def collate(self, indices, lg_offset: str = "num_nodes") -> Batch:
        """Batch of the given graphs, assembled on the device (same tensors as
        ``Batch.from_data_list([graphs...], lg_offset)``)."""
        pl = self.plan(indices, lg_offset)
        G = len(pl.idx)
        dev = next(iter(self.arrays.values())).device
        # one upload of every per-graph int64 offset array
        order = list(pl.fields.items())
        host = []
        for f, ent in order:
            host += [ent["src"], ent["dst"], ent["count"]]
            if "add" in ent:
                host.append(ent["add"])
        host += [pl.node_dst, pl.nodes, pl.ptr]
        flat = np.concatenate(host).astype(np.int64)
        staged = torch.from_numpy(flat)
        if dev.type == "cuda":
            staged = staged.pin_memory()
        offs = staged.to(dev, non_blocking=True)
        views, o = [], 0
        for h in host:
            views.append(offs[o:o + len(h)])
            o += len(h)
        lib = _lib.lib()
        s = stream_ptr()
        b = Batch()
        vi = 0
        for f, ent in order:
            src, dst, cnt = views[vi], views[vi + 1], views[vi + 2]
            vi += 3
            m = self.meta[f]
            a = self.arrays[f]
            if m["kind"] == "index":
                add = views[vi]
                vi += 1
                out = torch.empty(2, ent["total"], dtype=torch.int64, device=dev)
                _lib.check(lib.alignn_collate_index_i64(G, a.data_ptr(), a.size(1), src.data_ptr(), dst.data_ptr(),
                                                        cnt.data_ptr(), add.data_ptr(), ent["max"], out.data_ptr(),
                                                        out.size(1), s), "alignn_collate_index_i64")
            else:
                w = int(m.get("width", 1))
                out = torch.empty(ent["total"], w, dtype=torch.float32, device=dev)
                _lib.check(lib.alignn_collate_rows_f32(G, a.data_ptr(), w, src.data_ptr(), dst.data_ptr(),
                                                       cnt.data_ptr(), ent["max"], out.data_ptr(), s),
                           "alignn_collate_rows_f32")
                shape = m["shape"]
                out = out.view(ent["total"], *shape) if shape else out.view(ent["total"])
            setattr(b, f, out)
        node_dst, nodes, ptr = views[vi], views[vi + 1], views[vi + 2]
        batch = torch.empty(int(pl.nodes.sum()), dtype=torch.int64, device=dev)
        _lib.check(lib.alignn_collate_batchvec(G, node_dst.data_ptr(), nodes.data_ptr(), int(pl.nodes.max()),
                                               batch.data_ptr(), s), "alignn_collate_batchvec")
        b.batch = batch
        b.ptr = ptr.clone()
        b.num_graphs = G
        for k, vals in self.extras.items():
            setattr(b, k, [vals[i] for i in pl.idx])
        b._staging = (staged, offs)  # keep the pinned source alive until the copy has run
        return b
