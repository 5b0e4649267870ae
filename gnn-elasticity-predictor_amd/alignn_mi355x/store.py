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

The reference's per-sample transform (``PtGraphDataset``, ``scripts/train.py:49-216``) is part of the
store: graphs holding a NaN or an infinity in any float field are dropped when the store is built
(``_is_valid``, train.py:174-182; checked on the device, one launch per field), dataset indices count
the kept graphs only (train.py:64-87), the node features are cut to the scalar block without
mat2vec, padded or truncated to ``force_node_dim`` (train.py:103-117, :137-154), and once
:meth:`GraphStore.set_feature_standardization` has statistics the node scalars, mat2vec block and
global scalars are z-scored (train.py:184-216).  The transform runs inside the collate copy
(``alignn_collate_rows_std_f32``), so it costs no extra pass; :meth:`GraphStore.feature_stats`
computes the statistics over a training selection like train.py:1324-1380 (fp64 sums on the device).

On disk: a directory of ``<field>.npy`` arrays plus ``meta.json`` (no pickles; loaded with
``numpy.load(mmap_mode='r')``), written by :meth:`GraphStore.save`.
"""
from __future__ import annotations

import json
import os
import warnings
from dataclasses import dataclass
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


# ------------------------------------------------------------------------------------------------
# Fixed-capacity batches: a captured training plan (trainer.FusedTrainer) holds every size its
# launches were recorded with, so batches of real, variable-size crystals would each need a new plan.
# Instead a batch is padded to a capacity with one inert "ghost" graph: ghost atoms, ghost bonds in a
# ring over the ghost atoms, ghost triplets in a ring over a few ghost bonds (in-degrees below the
# attention kernels' heavy threshold), zero features; under the PyG offset rule the compacted line
# graph is filled up to the capacity with further ghost bonds (engine.BatchCache).  The ghost graph
# is disconnected from the real ones and its heads get no loss gradient, so every real output and
# gradient is the unpadded batch's (up to the summation order of reductions over rows); every padded
# batch has the capacity's sizes, i.e. one plan signature.
# ------------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class BatchCapacity:
    graphs: int                    # real graphs per batch (the ghost graph is one more)
    nodes: int                     # atoms, ghost atoms included
    edges: int                     # bonds
    triplets: int                  # line-graph edges
    active: Optional[int] = None   # compacted line-graph nodes (PyG offset rule); None: no compaction
    max_in_degree: int = 200       # of a ghost node (below SchedulePolicy.heavy_threshold = 256)


def ghost_plan(cap: BatchCapacity, B: int, N: int, E: int, T: int) -> Optional[Dict[str, int]]:
    """Ghost sizes padding a batch of B graphs with N atoms / E bonds / T triplets to ``cap``, or None
    when it does not fit: ga ghost atoms (>= 1), ge ghost bonds (ring over the ghost atoms), gt ghost
    triplets (ring over the first kg ghost bonds)."""
    if B != cap.graphs:
        return None
    ga, ge, gt = cap.nodes - N, cap.edges - E, cap.triplets - T
    if ga < 1 or ge < 0 or gt < 0:
        return None
    d = cap.max_in_degree
    if ge and -(-ge // ga) > d:
        return None
    kg = 0
    if gt:
        if ge == 0:
            return None
        kg = min(ge, max(1, -(-gt // d)))
        if -(-gt // kg) > d:
            return None
    return {"ga": ga, "ge": ge, "gt": gt, "kg": kg, "N": N, "E": E, "T": T}


def ghost_edges_host(count: int, base: int, mod: int) -> np.ndarray:
    """Host restatement of alignn_ghost_edges_i64 (tests): [2, count] ring edges."""
    j = np.arange(count, dtype=np.int64)
    return np.stack([base + (j + 1) % max(mod, 1), base + j % max(mod, 1)]) if count else np.zeros((2, 0), np.int64)


# PtGraphDataset's float fields checked by _is_valid (train.py:176)
VALIDATED_FIELDS = ("x", "edge_attr", "lg_edge_attr", "global_x", "sg_one_hot", "y")
BASE_SCALAR_DIM = 6   # train.py:102


class GraphStore:
    def __init__(self, arrays: Dict[str, torch.Tensor], counts: Dict[str, np.ndarray], meta: Dict,
                 extras: Optional[Dict[str, List]] = None, *, drop_invalid: bool = True, use_mat2vec: bool = True,
                 force_node_dim: Optional[int] = None):
        self.arrays = arrays          # field -> device tensor ([total, width] float32 or [2, total] int64)
        self.counts = counts          # field -> int64 [stored graphs] rows per graph
        self.meta = meta              # field -> {"kind": "rows"|"index", "shape": trailing shape}
        self.starts = {f: _excl_cumsum(c) for f, c in counts.items()}
        self.extras = extras or {}    # non-tensor per-graph attributes (e.g. material ids)
        self.num_stored = len(next(iter(counts.values())))
        self._staging = None
        self._stage_ring = []   # pinned host staging slots for collate's offset upload: [tensor, event]
        self._stage_next = 0
        # dataset index -> stored graph (graphs with NaN / inf dropped, as PtGraphDataset's file list)
        self.ids = self._valid_ids() if drop_invalid else np.arange(self.num_stored, dtype=np.int64)
        self.num_graphs = len(self.ids)
        if self.num_graphs == 0:
            raise ValueError("Dataset is empty after filtering for targets.")
        self._configure_nodes(use_mat2vec, force_node_dim)
        self._x_stats = None   # device (mean, std) over node_dim columns, identity where a block has none
        self._g_stats = None   # device (mean, std) over the global scalars
        # every stored graph's index fields point inside the graph (checked once here): batches collated
        # from the store then need no per-batch index validation (engine.prepare_batch skips its syncs)
        self.indices_checked = self._index_ranges_ok()

    # -------------------------------------------------------------------------------- capacity
    def field_kind(self, f: str) -> str:
        """'node' / 'edge' / 'triplet' (rows per graph = its atoms / bonds / line-graph edges) or
        'graph' (the same number of rows for every graph: global_x, sg_one_hot, y)."""
        named = {"x": "node", "edge_index": "edge", "edge_attr": "edge", "lg_edge_index": "triplet",
                 "lg_edge_attr": "triplet"}
        if f in named:
            return named[f]
        c = self.counts[f]
        if len(c) and np.all(c == c[0]):
            return "graph"
        for kind, ref in (("node", "x"), ("edge", "edge_index"), ("triplet", "lg_edge_index")):
            if ref in self.counts and np.array_equal(c, self.counts[ref]):
                return kind
        raise ValueError(f"field {f!r}: rows per graph follow neither atoms, bonds, triplets nor a constant")

    # index field -> the field whose rows it indexes (per graph: 0 <= index < that field's row count)
    INDEXED = {"edge_index": "x", "lg_edge_index": "edge_index"}

    def _index_ranges_ok(self) -> bool:
        """True when every index field is one of INDEXED and every stored graph's indices lie in
        [0, rows of the indexed field) — one pass per field on the stored arrays."""
        for f, m in self.meta.items():
            if m["kind"] != "index":
                continue
            ref = self.INDEXED.get(f)
            if ref is None or ref not in self.counts:
                return False
            a = self.arrays[f]
            cnt = self.counts[f]
            if a.numel() == 0:
                continue
            lim = self.counts[ref]   # rows (atoms) or index entries (bonds) per graph
            if a.device.type == "cuda":
                c = torch.from_numpy(cnt).to(a.device)
                lo = torch.segment_reduce(a.min(0).values.double(), "min", lengths=c, unsafe=True)
                hi = torch.segment_reduce(a.max(0).values.double(), "max", lengths=c, unsafe=True)
                lo, hi = lo.cpu().numpy(), hi.cpu().numpy()
            else:
                v = a.numpy()
                st = _excl_cumsum(cnt)
                nz = cnt > 0
                lo = np.zeros(len(cnt))
                hi = np.zeros(len(cnt))
                if nz.any():
                    lo[nz] = np.minimum.reduceat(v.min(0), st[nz])
                    hi[nz] = np.maximum.reduceat(v.max(0), st[nz])
            nz = cnt > 0
            if np.any(lo[nz] < 0) or np.any(hi[nz] >= lim[nz]):
                return False
        return True

    def _lg_spans(self) -> np.ndarray:
        """Per stored graph: [lo, hi] of its local line-graph endpoint ids (the bonds it touches lie
        inside), once, on the device."""
        if getattr(self, "_spans", None) is None:
            a = self.arrays["lg_edge_index"]
            cnt = torch.from_numpy(self.counts["lg_edge_index"]).to(a.device)
            lo = torch.segment_reduce(a.min(0).values.double(), "min", lengths=cnt, unsafe=True)
            hi = torch.segment_reduce(a.max(0).values.double(), "max", lengths=cnt, unsafe=True)
            self._spans = torch.stack([lo, hi], 1).cpu().numpy().astype(np.int64)
        return self._spans

    def _lg_bound_ok(self, gids: np.ndarray, lg_offset: str) -> bool:
        """Stored graphs ``gids`` collated in this order: every collated lg_edge_index entry (local
        index + PyG increment) is below the batch's bond count.  Implied for lg_offset='num_edges'."""
        if lg_offset != "num_nodes" or "lg_edge_index" not in self.counts:
            return True
        n, e, t = (self.counts[f][gids].astype(np.int64) for f in ("x", "edge_index", "lg_edge_index"))
        has = t > 0
        if not has.any():
            return True
        hi = (_excl_cumsum(n) + self._lg_spans()[gids][:, 1])[has]
        return int(hi.max()) < int(e.sum())

    def _deg_max(self) -> Dict[str, np.ndarray]:
        """Per stored graph: the largest in-degree of its atom graph ("ag": over its atoms) and of its
        line graph ("lg": over its local bond ids), once, on the device."""
        if getattr(self, "_degmax", None) is None:
            out = {}
            for f, rows in (("edge_index", "x"), ("lg_edge_index", "edge_index")):
                if f not in self.arrays or rows not in self.counts:
                    continue
                a = self.arrays[f]
                dev = a.device
                cnt = torch.from_numpy(self.counts[f]).to(dev)
                base = torch.repeat_interleave(torch.from_numpy(self.starts[rows]).to(dev), cnt,
                                               output_size=a.size(1))
                total = int(self.counts[rows].sum())
                deg = torch.bincount(a[1] + base, minlength=total)[:total]
                lens = torch.from_numpy(self.counts[rows]).to(dev)
                mx = torch.segment_reduce(deg.double(), "max", lengths=lens, unsafe=True) if total else deg.double()
                mx = torch.nan_to_num(mx, neginf=0.0).clamp(min=0.0)
                out["ag" if f == "edge_index" else "lg"] = mx.cpu().numpy().astype(np.int64)
            self._degmax = out
        return self._degmax

    def degree_bounds(self, gids: np.ndarray, lg_offset: str) -> Dict[str, int]:
        """Host bounds of every in-degree of a batch of stored graphs ``gids`` (collate order): the
        atom graph's is its graphs' largest; a line-graph bond's in-edges come from every graph whose
        shifted window [increment, increment + bonds) holds it — disjoint windows under
        lg_offset='num_edges', overlapping under PyG's 'num_nodes' rule — so its bound is the largest
        sum of window maxima over any point (a sweep over the window ends)."""
        dm = self._deg_max()
        out = {}
        if "ag" in dm:
            out["ag"] = int(dm["ag"][gids].max()) if len(gids) else 0
        if "lg" in dm:
            m = dm["lg"][gids]
            e = self.counts["edge_index"][gids].astype(np.int64)
            if lg_offset == "num_edges" or len(gids) == 0:
                out["lg"] = int(m.max()) if len(gids) else 0
            else:
                # each graph's in-edges land inside its touched-bond span [inc + lo, inc + hi] (the span
                # batch_sizes uses), not its whole window [inc, inc + bonds): tighter where windows overlap
                inc = _excl_cumsum(self.counts["x"][gids].astype(np.int64))
                t = self.counts["lg_edge_index"][gids].astype(np.int64)
                sp = self._lg_spans()[gids]
                has = t > 0
                inc, m, sp = inc[has], m[has], sp[has]
                if not has.any():
                    out["lg"] = 0
                    return out
                pos = np.concatenate([inc + sp[:, 0], inc + sp[:, 1] + 1])
                val = np.concatenate([m, -m])
                order = np.lexsort((val, pos))        # at one point, window ends (-) before starts (+)
                out["lg"] = int(max(0, np.cumsum(val[order]).max()))
        return out

    def batch_sizes(self, indices, lg_offset: str = "num_nodes") -> Dict[str, int]:
        """Host sizes of a batch: atoms, bonds, triplets, and an upper bound of the line graph's active
        bonds (union of each graph's touched-bond span shifted by its PyG increment)."""
        gids = self.ids[np.asarray(indices, dtype=np.int64)]
        n, e, t = (self.counts[f][gids].astype(np.int64) for f in ("x", "edge_index", "lg_edge_index"))
        inc = _excl_cumsum(n if lg_offset == "num_nodes" else e)
        sp = self._lg_spans()[gids]
        has = t > 0
        lo, hi = (inc + sp[:, 0])[has], (inc + sp[:, 1])[has]
        order = np.argsort(lo, kind="stable")
        lo, hi = lo[order], hi[order]
        # union length of the spans: each adds what lies beyond the furthest end before it
        prev = np.concatenate([[-1], np.maximum.accumulate(hi)[:-1]]) if len(hi) else hi
        active = int(np.maximum(0, hi - np.maximum(lo, prev + 1) + 1).sum()) if len(hi) else 0
        return {"nodes": int(n.sum()), "edges": int(e.sum()), "triplets": int(t.sum()), "active": active}

    def fits(self, indices, capacity: BatchCapacity, lg_offset: str = "num_nodes") -> Optional[Dict[str, int]]:
        """The ghost plan padding this batch to ``capacity``, or None when it does not fit (then the
        batch runs uncaptured).  With a compacted capacity the batch's active bonds (real ones — at most
        the span bound of batch_sizes — plus the kg ghost bonds its ghost triplets use) must not
        exceed ``capacity.active``; the compaction then marks inactive bonds (unused ghost bonds first,
        then real bonds without line-graph edges: engine.BatchCache._fill_active) until exactly
        ``capacity.active`` are active, which every batch of ``capacity.edges`` >= that many bonds allows."""
        sz = self.batch_sizes(indices, lg_offset)
        gp = ghost_plan(capacity, len(np.asarray(indices).reshape(-1)), sz["nodes"], sz["edges"], sz["triplets"])
        if gp is None or capacity.active is None:
            return gp
        if sz["active"] + gp["kg"] > capacity.active or capacity.active > capacity.edges:
            return None
        return gp

    def capacity(self, graphs: int, lg_offset: str = "num_nodes", samples: int = 512, margin: float = 0.02,
                 seed: int = 0, compact_fraction: float = 0.75) -> BatchCapacity:
        """A capacity that random batches of ``graphs`` dataset graphs fit (the largest of ``samples``
        random batches plus ``margin``, plus ghost room); rare larger batches run uncaptured."""
        rng = np.random.default_rng(seed)
        sz = [self.batch_sizes(rng.choice(self.num_graphs, size=graphs, replace=graphs > self.num_graphs), lg_offset)
              for _ in range(samples)]
        col = {k: np.asarray([z[k] for z in sz], dtype=np.int64) for k in sz[0]}
        grow = lambda v, extra: int(np.ceil(v * (1.0 + margin))) + extra  # noqa: E731
        nodes, edges, trip = grow(col["nodes"].max(), 4), grow(col["edges"].max(), 16), grow(col["triplets"].max(), 16)
        # the compacted line graph must hold each batch's active bonds plus the ghost bonds its ghost
        # triplets use (more for smaller batches: more ghost triplets)
        d = BatchCapacity.max_in_degree
        act = grow(int((col["active"] + -(-(trip - col["triplets"]) // d)).max()), 8)
        active = act if act <= compact_fraction * edges else None
        return BatchCapacity(graphs, nodes, edges, trip, active)

    # -------------------------------------------------------------------------------- transform
    def _configure_nodes(self, use_mat2vec: bool, force_node_dim: Optional[int]) -> None:
        """PtGraphDataset.__init__'s node-dimension rules (train.py:95-117)."""
        w = int(self.meta["x"].get("width", 1))
        self.raw_node_dim = w
        self.scalar_dim = min(BASE_SCALAR_DIM, w)
        raw_m2v = max(0, w - self.scalar_dim)
        self.use_mat2vec = bool(use_mat2vec)
        self.mat2vec_dim = raw_m2v if self.use_mat2vec else 0
        if force_node_dim is not None:
            force_node_dim = int(force_node_dim)
            if force_node_dim < self.scalar_dim:
                raise ValueError(f"Forced node dimension {force_node_dim} is smaller than scalar dimension "
                                 f"{self.scalar_dim}.")
            self.mat2vec_dim = max(force_node_dim - self.scalar_dim, 0)
            self.use_mat2vec = self.mat2vec_dim > 0
        self.node_dim = self.scalar_dim + self.mat2vec_dim
        # columns taken from a stored row (train.py:139-153): the scalar block alone without mat2vec,
        # then pad with zeros or truncate to node_dim
        sel = self.scalar_dim if (not self.use_mat2vec and raw_m2v > 0) else w
        self._x_copy_w = min(sel, self.node_dim)
        g = self.meta.get("global_x")
        self.global_scalar_dim = 0 if g is None else int(self.counts["global_x"][self.ids[0]]) * int(g.get("width", 1))

    def set_feature_standardization(self, scalar_mean=None, scalar_std=None, embed_mean=None, embed_std=None,
                                    global_mean=None, global_std=None) -> None:
        """PtGraphDataset.set_feature_standardization (train.py:184-198): z-score statistics applied by
        every later collate (None: that block is left as is)."""
        dev = next(iter(self.arrays.values())).device

        def vec(t, n, what):
            t = torch.as_tensor(t, dtype=torch.float32).reshape(-1)
            if t.numel() != n:
                raise ValueError(f"{what}: {t.numel()} statistics for {n} features")
            return t

        mean = torch.zeros(self.node_dim)
        std = torch.ones(self.node_dim)
        have = False
        if self.scalar_dim > 0 and scalar_mean is not None and scalar_std is not None:
            mean[:self.scalar_dim] = vec(scalar_mean, self.scalar_dim, "scalar_mean")
            std[:self.scalar_dim] = vec(scalar_std, self.scalar_dim, "scalar_std")
            have = True
        if self.mat2vec_dim > 0 and embed_mean is not None and embed_std is not None:
            mean[self.scalar_dim:] = vec(embed_mean, self.mat2vec_dim, "embed_mean")
            std[self.scalar_dim:] = vec(embed_std, self.mat2vec_dim, "embed_std")
            have = True
        # (v - 0) / 1 == v exactly, so a block without statistics passes through unchanged
        self._x_stats = (mean.to(dev), std.to(dev)) if have else None
        if self.global_scalar_dim > 0 and global_mean is not None and global_std is not None:
            self._g_stats = (vec(global_mean, self.global_scalar_dim, "global_mean").to(dev),
                             vec(global_std, self.global_scalar_dim, "global_std").to(dev))
        else:
            self._g_stats = None

    def feature_stats(self, train_idx, eps: float = 1e-12) -> Dict[str, Optional[torch.Tensor]]:
        """The reference's standardization statistics over the training graphs (train.py:1324-1380),
        from the features as a dataset item yields them before standardization: per-graph fp64 sums
        on the device accumulated in ``train_idx`` order, then mean, clamped variance and std in fp64,
        returned as fp32 host tensors (keys as the reference's scaler_state)."""
        idx = np.asarray(train_idx, dtype=np.int64).reshape(-1)
        gids = self.ids[idx]
        out: Dict[str, Optional[torch.Tensor]] = {k: None for k in ("scalar_mean", "scalar_std", "embed_mean",
                                                                     "embed_std", "global_mean", "global_std")}
        if len(gids) == 0:
            return out
        total_nodes = int(self.counts["x"][gids].sum())

        def sums(field, K, by_row):
            a = self.arrays[field]
            w = int(self.meta[field].get("width", 1))
            dev = a.device
            st = torch.from_numpy(np.stack([self.starts[field][gids], self.counts[field][gids]])).to(dev)
            lib = _lib.lib()
            ws = torch.empty(max(1, int(lib.alignn_feature_stats_workspace(len(gids), K))), dtype=torch.float64,
                             device=dev)
            sm = torch.empty(max(K, 1), dtype=torch.float64, device=dev)
            sq = torch.empty(max(K, 1), dtype=torch.float64, device=dev)
            _lib.check(lib.alignn_feature_stats_f64(len(gids), a.data_ptr(), w, st[0].data_ptr(), st[1].data_ptr(),
                                                    K, int(by_row), sm.data_ptr(), sq.data_ptr(), ws.data_ptr(),
                                                    ws.numel(), stream_ptr()), "alignn_feature_stats_f64")
            return sm[:K].cpu().numpy(), sq[:K].cpu().numpy()

        if total_nodes > 0:
            s_all = np.zeros(self.node_dim)
            q_all = np.zeros(self.node_dim)
            if self._x_copy_w > 0:
                s_all[:self._x_copy_w], q_all[:self._x_copy_w] = sums("x", self._x_copy_w, False)
            for name, lo, hi in (("scalar", 0, self.scalar_dim), ("embed", self.scalar_dim, self.node_dim)):
                if hi <= lo:
                    continue
                mean = s_all[lo:hi] / total_nodes
                var = np.maximum(q_all[lo:hi] / total_nodes - mean ** 2, eps)
                out[f"{name}_mean"] = torch.from_numpy(mean.astype(np.float32))
                out[f"{name}_std"] = torch.from_numpy(np.sqrt(var).astype(np.float32))
        if self.global_scalar_dim > 0:
            s, q = sums("global_x", self.global_scalar_dim, True)
            mean = s / len(gids)
            var = np.maximum(q / len(gids) - mean ** 2, eps)
            out["global_mean"] = torch.from_numpy(mean.astype(np.float32))
            out["global_std"] = torch.from_numpy(np.sqrt(var).astype(np.float32))
        return out

    def _valid_ids(self) -> np.ndarray:
        """Stored graphs without NaN / inf in any checked float field (device check, one launch per field)."""
        dev = next(iter(self.arrays.values())).device
        G = self.num_stored
        if dev.type != "cuda":   # a host-side store (save / load round trips): the same rule in numpy
            ok = np.ones(G, dtype=bool)
            for f in VALIDATED_FIELDS:
                if f in self.arrays and self.meta[f]["kind"] == "rows" and self.arrays[f].numel():
                    w = int(self.meta[f].get("width", 1))
                    fin = np.isfinite(self.arrays[f].numpy().reshape(-1, w)).all(axis=1)
                    bad = np.add.reduceat(~fin, self.starts[f]) if len(fin) else np.zeros(G, dtype=int)
                    ok &= (bad == 0) | (self.counts[f] == 0)
            return np.nonzero(ok)[0].astype(np.int64)
        ok = torch.ones(max(G, 1), dtype=torch.int32, device=dev)
        lib = _lib.lib()
        for f in VALIDATED_FIELDS:
            if f not in self.arrays or self.meta[f]["kind"] != "rows":
                continue
            a = self.arrays[f]
            w = int(self.meta[f].get("width", 1))
            if a.dtype != torch.float32 or a.numel() == 0:
                continue
            st = torch.from_numpy(np.stack([self.starts[f], self.counts[f]])).to(dev)
            _lib.check(lib.alignn_segment_finite_f32(G, a.data_ptr(), w, st[0].data_ptr(), st[1].data_ptr(),
                                                     int(self.counts[f].max()) if G else 0, ok.data_ptr(),
                                                     stream_ptr()), "alignn_segment_finite_f32")
        return np.nonzero(ok[:G].cpu().numpy())[0].astype(np.int64)

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
                if key in ("global_x", "sg_one_hot"):
                    # a column per graph (train.py:164-169): fetch.to_pyg_data stores [1, 59] / [1, 230]
                    vals = [v.reshape(-1, 1) for v in vals]
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
    def from_data_list(cls, data_list: Sequence[Data], device, require_target: bool = True, **kw) -> "GraphStore":
        """kw: drop_invalid, use_mat2vec, force_node_dim (PtGraphDataset's options, train.py:50-57).
        require_target: graphs without ``y`` are skipped (train.py:74-75)."""
        if require_target:
            data_list = [d for d in data_list if getattr(d, "y", None) is not None]
        arrays, counts, meta, extras = cls.host_arrays(data_list)
        dev = {k: torch.from_numpy(np.ascontiguousarray(v)).to(device) for k, v in arrays.items()}
        return cls(dev, counts, meta, extras, **kw)

    def save(self, path: str) -> None:
        os.makedirs(path, exist_ok=True)
        for k, v in self.arrays.items():
            np.save(os.path.join(path, f"{k}.npy"), v.cpu().numpy())
            np.save(os.path.join(path, f"{k}.counts.npy"), self.counts[k])
        with open(os.path.join(path, "meta.json"), "w") as f:
            json.dump({"fields": self.meta, "extras": {k: [str(x) for x in v] for k, v in self.extras.items()}}, f)

    @classmethod
    def load(cls, path: str, device, **kw) -> "GraphStore":
        with open(os.path.join(path, "meta.json")) as f:
            m = json.load(f)
        arrays, counts = {}, {}
        for k in m["fields"]:
            a = np.load(os.path.join(path, f"{k}.npy"), mmap_mode="r")      # no pickles
            with warnings.catch_warnings():   # a read-only map: .to(device) copies, nothing writes it
                warnings.simplefilter("ignore", UserWarning)
                arrays[k] = torch.from_numpy(np.ascontiguousarray(a)).to(device)
            counts[k] = np.load(os.path.join(path, f"{k}.counts.npy"))
        return cls(arrays, counts, m["fields"], m.get("extras", {}), **kw)

    # -------------------------------------------------------------------------------- batches
    def plan(self, indices, lg_offset: str = "num_nodes") -> CollatePlan:
        """indices: dataset indices (over the kept graphs)."""
        idx = np.asarray(indices, dtype=np.int64).reshape(-1)
        if idx.size == 0:
            raise ValueError("cannot collate an empty list")
        if idx.min() < 0 or idx.max() >= self.num_graphs:
            raise IndexError("graph index out of range")
        pl = CollatePlan(self.meta, self.counts, self.starts, self.ids[idx], lg_offset)
        pl.sample_index = idx
        return pl

    STAGE_SLOTS = 8

    def _stage_slot(self, src: torch.Tensor):
        """``src`` copied into the next pinned staging slot (grown, never shrunk): a ring of pinned host
        buffers reused batch after batch, so collate allocates no pinned memory per batch (a pinned
        allocation can wait for the device).  A slot is reused after the upload that read it ran."""
        n = src.numel()
        if len(self._stage_ring) < self.STAGE_SLOTS:
            self._stage_ring.append([torch.empty(0, dtype=torch.int64).pin_memory(), torch.cuda.Event()])
        slot = self._stage_ring[self._stage_next % len(self._stage_ring)]
        self._stage_next += 1
        slot[1].synchronize()   # the upload that last read this slot (long done but for 8 batches in flight)
        if slot[0].numel() < n:
            slot[0] = torch.empty(max(n, 2 * slot[0].numel()), dtype=torch.int64).pin_memory()
        buf = slot[0][:n]
        buf.copy_(src)
        return buf, slot[1]

    def collate(self, indices, lg_offset: str = "num_nodes", capacity: Optional[BatchCapacity] = None) -> Batch:
        """Batch of the given graphs, assembled on the device (same tensors as
        ``Batch.from_data_list([graphs...], lg_offset)``).  With a ``capacity`` the batch is padded
        to it by one ghost graph (``num_real_graphs`` = the real graph count); a batch that does not
        fit is returned unpadded."""
        pl = self.plan(indices, lg_offset)
        sample_index_np = pl.sample_index
        G = len(pl.idx)
        dev = next(iter(self.arrays.values())).device
        gh = None
        if capacity is not None and "lg_edge_index" in pl.fields:
            gh = self.fits(indices, capacity, lg_offset)
        if gh is not None:   # the ghost graph's atoms in the batch vector and ptr
            pl.node_dst = np.append(pl.node_dst, gh["N"])
            pl.nodes = np.append(pl.nodes, gh["ga"])
            pl.ptr = np.append(pl.ptr, capacity.nodes)
        # one upload of every per-graph int64 offset array
        order = list(pl.fields.items())
        host = []
        for f, ent in order:
            host += [ent["src"], ent["dst"], ent["count"]]
            if "add" in ent:
                host.append(ent["add"])
        host += [pl.node_dst, pl.nodes, pl.ptr, pl.sample_index]
        flat = np.concatenate(host).astype(np.int64)
        staged = torch.from_numpy(flat)
        if dev.type == "cuda":
            staged, ev = self._stage_slot(staged)
            offs = staged.to(dev, non_blocking=True)
            ev.record(torch.cuda.current_stream(dev))   # the slot is free again once the copy has read it
        else:
            offs = staged.to(dev)
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
            rows = ent["total"]
            if gh is not None:
                kind = self.field_kind(f)
                rows = {"node": capacity.nodes, "edge": capacity.edges, "triplet": capacity.triplets,
                        "graph": ent["total"] + (ent["total"] // G if G else 0)}[kind]
            if m["kind"] == "index":
                add = views[vi]
                vi += 1
                out = torch.empty(2, rows, dtype=torch.int64, device=dev)
                _lib.check(lib.alignn_collate_index_i64(G, a.data_ptr(), a.size(1), src.data_ptr(), dst.data_ptr(),
                                                        cnt.data_ptr(), add.data_ptr(), ent["max"], out.data_ptr(),
                                                        out.size(1), s), "alignn_collate_index_i64")
                if gh is not None:   # ghost bonds: ring over the ghost atoms; ghost triplets: over kg ghost bonds
                    base, mod = (gh["N"], gh["ga"]) if kind == "edge" else (gh["E"], gh["kg"])
                    _lib.check(lib.alignn_ghost_edges_i64(out.data_ptr(), out.size(1), ent["total"],
                                                          rows - ent["total"], base, mod, s), "alignn_ghost_edges_i64")
            else:
                w = int(m.get("width", 1))
                ow, copy_w, stats, by_row = w, w, None, 0
                if f == "x":
                    ow, copy_w, stats = self.node_dim, self._x_copy_w, self._x_stats
                elif f == "global_x":
                    stats, by_row = self._g_stats, 1
                out = torch.empty(rows, ow, dtype=torch.float32, device=dev)
                if rows > ent["total"]:   # ghost rows: zero features, target 1 (positive for the log transform)
                    _lib.check(lib.alignn_fill_f32(out[ent["total"]:].data_ptr(), (rows - ent["total"]) * ow,
                                                   1.0 if f == "y" else 0.0, s), "alignn_fill_f32")
                if (ow, copy_w, stats) == (w, w, None):
                    _lib.check(lib.alignn_collate_rows_f32(G, a.data_ptr(), w, src.data_ptr(), dst.data_ptr(),
                                                           cnt.data_ptr(), ent["max"], out.data_ptr(), s),
                               "alignn_collate_rows_f32")
                else:   # PtGraphDataset.__getitem__'s select / pad / truncate / z-score, fused
                    _lib.check(lib.alignn_collate_rows_std_f32(
                        G, a.data_ptr(), w, src.data_ptr(), dst.data_ptr(), cnt.data_ptr(), ent["max"],
                        out.data_ptr(), ow, copy_w, None if stats is None else stats[0].data_ptr(),
                        None if stats is None else stats[1].data_ptr(), by_row, s), "alignn_collate_rows_std_f32")
                shape = m["shape"] if ow == w else [ow]
                out = out.view(rows, *shape) if shape else out.view(rows)
            setattr(b, f, out)
        node_dst, nodes, ptr, sample_index = views[vi], views[vi + 1], views[vi + 2], views[vi + 3]
        batch = torch.empty(int(pl.nodes.sum()), dtype=torch.int64, device=dev)
        _lib.check(lib.alignn_collate_batchvec(len(pl.nodes), node_dst.data_ptr(), nodes.data_ptr(),
                                               int(pl.nodes.max()), batch.data_ptr(), s), "alignn_collate_batchvec")
        b.batch = batch
        # index ranges checked at build (no per-batch sync).  Each graph's local indices lie below its
        # own row counts; the collated line-graph index (+ the PyG increment) must also lie below the
        # batch's bond count, which lg_offset='num_nodes' does not imply (a graph with fewer bonds than
        # atoms): checked here on the host from the per-graph spans
        b._alignn_trusted = self.indices_checked and self._lg_bound_ok(pl.idx, lg_offset)
        if b._alignn_trusted:
            # host facts that let engine.BatchCache prepare the batch without a device->host copy: in-degree
            # bounds (device-built attention schedules) and, unpadded under PyG's offset rule, the size of
            # the compacted line graph (the span bound of batch_sizes; inert bonds fill it up)
            hints = self.degree_bounds(pl.idx, lg_offset)
            if gh is not None:
                hints = {k: max(v, capacity.max_in_degree) for k, v in hints.items()}
            elif lg_offset == "num_nodes" and "lg_edge_index" in pl.fields:
                hints["lg_active"] = self.batch_sizes(sample_index_np, lg_offset)["active"]
            b._alignn_hints = hints
        b.ptr = ptr.clone()
        b.sample_index = sample_index.clone()   # train.py:171 (dataset indices of the batch's graphs)
        b.num_graphs = G
        if gh is not None:
            b.num_graphs = G + 1
            b.num_real_graphs = G
            # read by engine.BatchCache: ghost bonds after the first kg fill the compacted line graph
            b._alignn_pad = {"edges": gh["E"], "kg": gh["kg"], "active": capacity.active}
        for k, vals in self.extras.items():
            setattr(b, k, [vals[i] for i in pl.idx])
        b._staging = (staged, offs)  # keep the pinned source alive until the copy has run
        return b
