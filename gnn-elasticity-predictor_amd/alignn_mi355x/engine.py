"""ALIGNN forward/backward engine over libalignn_hip (MI355X, fp32).

One call of :meth:`AlignnEngine.forward` runs the whole ``HeteroAlignnRegressor.forward``
(``scripts/train.py:537-586``); :meth:`AlignnEngine.backward` produces every parameter gradient
into a flat buffer (layout: :mod:`layout`).  All arithmetic is in HIP kernels: MFMA GEMMs for the
dense projections, fused CSR attention kernels for TransformerConv message passing, fused row
kernels for gate/LayerNorm/ReLU/dropout/residual and readout.  Torch supplies memory and the stream.

Data layout in HBM (D = hidden, H = heads, C = D/H):
  * node/edge state    [N, D] / [E, D] row-major fp32
  * QKVR               [n, 4D]   (Q | K | V | R=skip) of each TransformerConv
  * U, S, Vd, Sz       [n, H, D] per-target-node per-head vectors of the edge-feature algebra
  * angle embedding    [T, D]    in line-graph target-sorted order (coalesced per segment)
  * CSR                int32 offsets/permutations per graph (ops.GraphCSR)
"""
from __future__ import annotations

from contextlib import contextmanager
from typing import Dict, List, Optional

import numpy as np
import torch

from . import ops
from .layout import AlignnConfig, offsets

MIN_LOGVAR_FLOOR = -2.9  # train.py:39


# ------------------------------------------------------------------------------------------------
# Parameter / gradient views over a flat buffer
# ------------------------------------------------------------------------------------------------
class _Conv:
    __slots__ = ("Wqkvr", "bqkvr", "We", "wbeta", "lnw", "lnb", "Wp", "bp")


class FlatViews:
    """Named views (state-dict names) + fused operand views of one flat fp32 buffer."""

    def __init__(self, flat: torch.Tensor, cfg: AlignnConfig, hetero: bool = True):
        self.flat = flat
        self.cfg = cfg
        self.hetero = hetero
        self.prefix = pre = "base." if hetero else ""
        offs, total, self.sigma_start = offsets(cfg, hetero)
        if flat.numel() != total:
            raise ValueError(f"flat buffer has {flat.numel()} elements, layout needs {total}")
        self.named: Dict[str, torch.Tensor] = {}
        for name, (o, shape) in offs.items():
            n = 1
            for s in shape:
                n *= s
            self.named[name] = flat[o:o + n].view(shape)
        D = cfg.hidden
        self.edge: List[_Conv] = [self._conv(f"{pre}edge_blocks.{l}.", offs, D, False) for l in range(cfg.layers)]
        self.node: List[_Conv] = [self._conv(f"{pre}node_blocks.{l}.", offs, D, True) for l in range(cfg.layers)]
        self.edge_We = self._stack(offs, "edge_blocks.{}.conv.lin_edge.weight", (D, D))
        self.node_We = self._stack(offs, "node_blocks.{}.conv.lin_edge.weight", (D, D))
        self.node_Wp = self._stack(offs, "node_blocks.{}.edge_proj.weight", (D, D))
        self.node_bp = self._stack(offs, "node_blocks.{}.edge_proj.bias", (D,))
        # [L, 4D, D] stacks of each conv's [Wq; Wk; Wv; Wskip] block
        self.edge_Wqkvr = self._stack(offs, "edge_blocks.{}.conv.lin_query.weight", (4 * D, D))
        self.node_Wqkvr = self._stack(offs, "node_blocks.{}.conv.lin_query.weight", (4 * D, D))
        T = cfg.target_dim

        def rows(name, k):
            o = offs[name][0]
            return flat[o:o + k * D].view(k, D) if k * D else None

        def vec(name, k):
            o = offs[name][0]
            return flat[o:o + k]

        if hetero:
            self.Wmean, self.bmean = rows("mean_heads.0.weight", T), vec("mean_heads.0.bias", T)
            self.Wlogvar, self.blogvar = rows("logvar_heads.0.weight", T), vec("logvar_heads.0.bias", T)
        else:
            self.Wout, self.bout = rows("output_heads.0.weight", T), vec("output_heads.0.bias", T)

    def _stack(self, offs, pattern: str, shape):
        """[L, *shape] strided view of one per-layer tensor (layers sit at a constant stride)."""
        L = self.cfg.layers
        if L == 0:
            return None
        o = [offs[self.prefix + pattern.format(l)][0] for l in range(L)]
        stride = o[1] - o[0] if L > 1 else 0
        if any(o[l] - o[0] != l * stride for l in range(L)):
            raise AssertionError("per-layer parameters are not equally spaced in the flat layout")
        inner = [1] * len(shape)
        for i in range(len(shape) - 2, -1, -1):
            inner[i] = inner[i + 1] * shape[i + 1]
        return self.flat.as_strided((L, *shape), (stride, *inner), self.flat.storage_offset() + o[0])

    def enc(self, which: str, idx: int, kind: str) -> torch.Tensor:
        return self.named[f"{self.prefix}{which}_encoder.{idx}.{kind}"]

    def _conv(self, p: str, offs, D: int, node: bool) -> _Conv:
        c = _Conv()
        o = offs[p + "conv.lin_query.weight"][0]
        c.Wqkvr = self.flat[o:o + 4 * D * D].view(4 * D, D)
        o = offs[p + "conv.lin_query.bias"][0]
        c.bqkvr = self.flat[o:o + 4 * D]
        c.We = self.named[p + "conv.lin_edge.weight"]
        c.wbeta = self.named[p + "conv.lin_beta.weight"].view(-1)
        c.lnw = self.named[p + "norm.weight"]
        c.lnb = self.named[p + "norm.bias"]
        c.Wp = self.named[p + "edge_proj.weight"] if node else None
        c.bp = self.named[p + "edge_proj.bias"] if node else None
        return c

    def __getitem__(self, name: str) -> torch.Tensor:
        return self.named[name]


# ------------------------------------------------------------------------------------------------
# Per-batch device preparation (cached on the batch)
# ------------------------------------------------------------------------------------------------
class BatchCache:
    """CSR lists of the atom graph and the line graph, target-sorted angle inputs, ptr."""

    # the atom graph's attention kernels take four targets per workgroup: XCD-contiguous item ranges
    # interleaved in chunks of four (1: one item at a time, as for the line graph)
    ATOM_XCD_CHUNK = 4

    def __init__(self, batch, validate: bool = True):
        # a batch collated from a GraphStore whose index ranges were checked when it was built needs
        # no per-batch check (two host syncs fewer)
        validate = validate and not getattr(batch, "_alignn_trusted", False)
        x = batch.x
        if not x.is_cuda:
            raise ValueError("batch must be on the HIP device (batch.to('cuda')); the engine has no CPU path")
        self.N = int(x.size(0))
        self.E = int(batch.edge_index.size(1))
        self.T = int(batch.lg_edge_index.size(1))
        # host facts of a batch collated from a GraphStore (store.collate): in-degree bounds (the
        # attention schedules are then built on the device) and the compacted line graph's size
        hints = getattr(batch, "_alignn_hints", None) or {}
        self.ag = ops.GraphCSR(batch.edge_index, self.N)
        self.ag.xcd_chunk = self.ATOM_XCD_CHUNK
        self.ag.deg_bound = hints.get("ag")
        if validate:
            self.ag.check_indices("edge_index")
        # a batch padded to a store.BatchCapacity: the ghost graph fills the compacted line graph up
        # to the capacity's size (and the loss covers the real graphs only, trainer)
        self.pad = getattr(batch, "_alignn_pad", None)
        self.real_graphs = getattr(batch, "num_real_graphs", None)
        self.lg = self._line_graph(batch.lg_edge_index, self.E, validate, self.pad, hints.get("lg_active"))
        self.lg.deg_bound = hints.get("lg")
        la = batch.lg_edge_attr
        self.angle_dim = int(la.size(-1)) if la.dim() == 2 else 0
        if self.T > 0 and la.numel() > 0:
            # target-sorted angle inputs, rows padded to a multiple of 4 floats (16-byte aligned rows:
            # the encoder GEMMs read them with float4 loads; the pad column is never read)
            a = la.contiguous().float()
            ld = (a.size(1) + 3) // 4 * 4
            buf = torch.empty(self.T, ld, device=a.device)
            self._xa_buf = buf
            self.xa = buf[:, :a.size(1)]
            ops.gather_rows(a, self.lg.perm_dst[: self.T], self.xa)
        else:
            self.xa = None
            self._xa_buf = None
        if hasattr(batch, "batch") and batch.batch is not None:
            self.batch_vec = batch.batch.to(torch.int64).contiguous()
        else:
            self.batch_vec = torch.zeros(self.N, dtype=torch.int64, device=x.device)
        if hasattr(batch, "ptr") and batch.ptr is not None:
            self.ptr = batch.ptr.to(torch.int64).contiguous()
        else:  # host logic (plumbing): counts per graph
            B = int(self.batch_vec.max().item()) + 1 if self.N else 0
            cnt = torch.bincount(self.batch_vec, minlength=B)
            self.ptr = torch.cat([cnt.new_zeros(1), cnt.cumsum(0)])
        self.B = int(self.ptr.numel() - 1)

    # -------------------------------------------------------------------------------------------
    # Re-binding a captured step to a new batch (FusedTrainer._rebind): a launch plan holds the
    # device addresses of its batch and of this cache, and the sizes every launch was recorded
    # with.  A new batch whose cache has the same signature (every size a recorded launch depends
    # on: node/edge/triplet counts, the compacted line graph's size, the schedules' list lengths and
    # flags) can be copied into the captured batch's buffers and the plan replayed unchanged.
    # -------------------------------------------------------------------------------------------
    def schedules(self) -> None:
        """Builds the atom and line graphs' schedules: on the device when the batch's in-degrees are
        bounded on the host (store batches, GraphCSR.device_schedule_ok), else with ONE device->host
        copy of both graphs' offsets (the in-degrees order the work items) instead of one per graph."""
        for g in (self.ag, self.lg):   # host-bounded in-degrees: built on the device, no copy
            if g._sched is None and g.device_schedule_ok():
                g.schedule()
        gs = [g for g in (self.ag, self.lg) if g._sched is None]
        if len(gs) == 2:
            off = torch.cat([g.off_dst for g in gs]).cpu().numpy().astype(np.int64)
            a = gs[0].n + 1
            for g, o in ((gs[0], off[:a]), (gs[1], off[a:])):
                g.schedule(deg=o[1:] - o[:-1] if g.n else np.zeros(0, np.int64))
        for g in (self.ag, self.lg):
            g.schedule()

    @staticmethod
    def _graph_sig(g: ops.GraphCSR):
        sc = g.schedule()
        return (g.n, g.m, g.n_full, g.rows is not None, int(sc.n_light), int(sc.n_heavy), int(sc.flags))

    def signature(self):
        return (self.N, self.E, self.T, self.B, self.real_graphs, self.angle_dim,
                None if self._xa_buf is None else tuple(self._xa_buf.shape),
                self._graph_sig(self.ag), self._graph_sig(self.lg),
                tuple(self.batch_vec.shape), tuple(self.ptr.shape))

    @staticmethod
    def _graph_tensors(g: ops.GraphCSR):
        g.schedule()
        _, light, heavy = g._sched
        return [g.off_dst, g.perm_dst, g.src_at, g.dst_at, g.off_src, g.pos_src, g.err, light, heavy, g.rows, g.cmap,
                g.dst_src()]

    def device_tensors(self):
        """Every device buffer of this cache, in a fixed order (None where absent)."""
        return self._graph_tensors(self.ag) + self._graph_tensors(self.lg) + [self._xa_buf, self.batch_vec, self.ptr]

    def copy_pairs(self, dst: "BatchCache"):
        """(dst buffer, this cache's buffer) pairs for a copy into ``dst`` (same signature)."""
        pairs = []
        for a, b in zip(self.device_tensors(), dst.device_tensors()):
            if (a is None) != (b is None):
                raise ValueError("batch caches of different structure")
            if a is not None and a.numel():
                if a.shape != b.shape or a.dtype != b.dtype:
                    raise ValueError(f"batch cache buffer {tuple(a.shape)} {a.dtype} vs {tuple(b.shape)} {b.dtype}")
                pairs.append((b, a))
        return pairs

    def copy_into(self, dst: "BatchCache") -> None:
        """dst's buffers <- this cache's contents (same signature; stream-ordered device copies)."""
        ops.copy_many(self.copy_pairs(dst))

    # A line-graph node (bond) with neither in- nor out-edges contributes nothing to the attention
    # (empty segment, never a source).  Under PyG's lg_edge_index offset rule most
    # bonds of a batch are such nodes (B=32: 2,580 of 23,040 active), so the line graph is re-indexed
    # over the active bonds and the per-node GEMMs of the line convs run on those rows only.
    COMPACT_FRACTION = 0.75

    @classmethod
    def _line_graph(cls, edge_index: torch.Tensor, n: int, validate: bool, pad=None,
                    active_bound: Optional[int] = None) -> ops.GraphCSR:
        """CSR of the line graph, compacted when few bonds are active.  The active set is marked from
        the edge endpoints directly (no CSR of all n bonds is built first): one CSR build per batch.
        pad (a padded batch): compaction as its capacity says; with a compacted capacity, ghost bonds
        past the first pad['kg'] (those the ghost triplets use) join the active set until it has
        pad['active'] members — device arithmetic, no host round trip.  active_bound (a host bound
        of the active count, store batches): the same filling up to that many, so the size needs no
        device->host copy either (a bond without line-graph edges is inert in the compacted graph).
        Equality with the unhinted step is bitwise only when the bound is exact (the synthetic MP-like
        batches: every bond of the span active); a looser bound adds inert rows, which change the
        compacted row count and with it split-K chunking and column-sum partitions, so the two agree to
        fp32 summation order (and COMPACT_FRACTION is decided on the bound)."""
        if edge_index.dtype != torch.int64 or edge_index.dim() != 2 or edge_index.size(0) != 2:
            raise ValueError("edge_index must be int64 [2, m]")
        m = edge_index.size(1)
        if n == 0 or m == 0:
            g = ops.GraphCSR(edge_index, n)
            if validate:
                g.check_indices("lg_edge_index")
            return g
        if validate:
            lo, hi = torch.stack([edge_index.min(), edge_index.max()]).tolist()
            if lo < 0 or hi >= n:
                raise IndexError(f"lg_edge_index: edge index out of range [0, {n})")
        if pad is not None and pad["active"] is None:
            return ops.GraphCSR(edge_index, n)
        if pad is None and active_bound is not None and not (0 < active_bound <= cls.COMPACT_FRACTION * n):
            return ops.GraphCSR(edge_index, n)
        active = torch.zeros(n, dtype=torch.bool, device=edge_index.device)
        active.index_fill_(0, edge_index[0], True)    # (index_fill_: no host sync, unlike index_put_)
        active.index_fill_(0, edge_index[1], True)
        if pad is not None:
            active = cls._fill_active(active, pad["edges"] + pad["kg"], int(pad["active"]))
            na = int(pad["active"])
        elif active_bound is not None:
            active = cls._fill_active(active, n, int(active_bound))
            na = int(active_bound)
        else:
            na = None
        return cls._compact(active, edge_index, n, force=na is not None, na=na)

    @staticmethod
    def _fill_active(active: torch.Tensor, first: int, na: int) -> torch.Tensor:
        """Marks inactive bonds until ``na`` are active (device arithmetic, no host round trip): the
        unused ghost bonds (index >= first) first, so the real rows keep their order and positions in
        every compacted product, then any other inactive bond — a bond without line-graph edges is an
        empty segment and never a source, so it is inert in the compacted graph.  The batch's real
        active count is only bounded on the host (store.batch_sizes); taking from every inactive bond
        keeps exactly ``na`` marked whenever n >= na, so the compaction's fixed-size index list
        (nonzero_static) is never padded with -1."""
        n = active.numel()
        inactive = ~active
        ghost = torch.arange(n, device=active.device) >= first
        need = na - active.sum()
        c1 = inactive & ghost
        take1 = c1 & (torch.cumsum(c1, 0) <= need)
        c2 = inactive & ~ghost
        take2 = c2 & (torch.cumsum(c2, 0) <= need - take1.sum())
        return active | take1 | take2

    @classmethod
    def _compact(cls, active: torch.Tensor, edge_index: torch.Tensor, n: int, force: bool = False,
                 na: Optional[int] = None) -> ops.GraphCSR:
        """na: the active count when the caller knows it (a padded batch: its capacity's), so neither
        the count nor the index list waits for the device."""
        if na is None:
            na = int(active.sum().item())
            if na > cls.COMPACT_FRACTION * n and not force:
                return ops.GraphCSR(edge_index, n)
            rows = torch.nonzero(active).flatten()
        else:
            rows = torch.nonzero_static(active, size=na).flatten()
        cmap = torch.full((n,), -1, dtype=torch.int64, device=edge_index.device)
        cmap[rows] = torch.arange(na, dtype=torch.int64, device=edge_index.device)
        gc = ops.GraphCSR(cmap[edge_index], na)
        gc.rows = rows.to(torch.int32)
        gc.n_full = n
        gc.cmap = cmap.to(torch.int32)
        return gc


def prepare_batch(batch, stream: Optional[torch.cuda.Stream] = None, validate: bool = True) -> BatchCache:
    """Builds the batch's device cache (CSR lists, line-graph compaction, schedules) on ``stream``
    (default: the current one) and records an event there that a step on another stream waits
    for (FusedTrainer.step): a loader can prepare batch i + 1 on its own stream while step i runs."""
    if stream is None:
        bc = batch_cache(batch, validate)
        bc.schedules()       # both graphs' schedules from one device->host copy of their offsets
        bc.device_tensors()  # and the by-source target lists
    else:
        with torch.cuda.stream(stream):
            bc = batch_cache(batch, validate)
            bc.schedules()
            bc.device_tensors()
    ev = torch.cuda.Event()
    s = stream if stream is not None else torch.cuda.current_stream()
    ev.record(s)
    try:
        batch._alignn_ready = ev
        batch._alignn_adopted = {s.cuda_stream}
    except AttributeError:
        pass
    return bc


def batch_cache(batch, validate: bool = True) -> BatchCache:
    """The batch's device cache (built on first use).  A batch prepared on another stream
    (:func:`prepare_batch`) is adopted by the current stream first: it waits for the preparation's
    event, and every buffer of the batch and its cache is marked as used here, so the caching
    allocator cannot hand them out again before this stream's reads ran — on every path that reads
    the batch (replay, re-binding, eager steps, the module API)."""
    bc = getattr(batch, "_alignn_cache", None)
    if bc is None:
        bc = BatchCache(batch, validate)
        try:
            batch._alignn_cache = bc
        except AttributeError:
            pass
    else:
        adopt(batch, bc)
    return bc


def adopt(batch, bc: Optional[BatchCache] = None) -> None:
    """Current stream waits for ``batch``'s preparation event and records its use of the batch's
    buffers (once per stream; no-op for batches prepared on the current stream or never prepared,
    and inside a graph capture, whose stream is ordered after the eager stream that adopted it)."""
    ev = getattr(batch, "_alignn_ready", None)
    if ev is None or torch.cuda.is_current_stream_capturing():
        return
    bc = bc if bc is not None else getattr(batch, "_alignn_cache", None)
    dev = batch.x.device
    s = torch.cuda.current_stream(dev)
    seen = batch.__dict__.setdefault("_alignn_adopted", set())
    if s.cuda_stream in seen:
        return
    seen.add(s.cuda_stream)
    s.wait_event(ev)
    tensors = [v for v in vars(batch).values() if torch.is_tensor(v)]
    if bc is not None:
        tensors += bc.device_tensors()
    for t in tensors:
        if t is not None and t.is_cuda:
            t.record_stream(s)


_PRIVATE_SKIP = ("_alignn_cache", "_alignn_ready", "_alignn_adopted", "_staging")


def clone_batch(batch):
    """A private copy of ``batch`` (its tensors cloned on the current stream; hints kept, device caches
    not): the buffers a recorded plan reads, so that re-binding other batches never writes the caller's."""
    out = type(batch).__new__(type(batch))
    for k, v in batch.__dict__.items():
        if k in _PRIVATE_SKIP:
            continue
        out.__dict__[k] = v.clone() if torch.is_tensor(v) else v
    return out


def batch_versions(batch, fields) -> tuple:
    """In-place modification counters of ``batch``'s fields (torch's tensor._version)."""
    return tuple(getattr(batch, k)._version if torch.is_tensor(getattr(batch, k, None)) else None for k in fields)


def site_seed(seed: int, site: int) -> int:
    return (seed * 0x9E3779B1 + site * 0x85EBCA77 + 0x165667B1) & (2**63 - 1)


class _Ctx:
    pass


# ------------------------------------------------------------------------------------------------
# One conv block (EdgeUpdateBlock / NodeUpdateBlock) — shared by the full engine and the
# standalone drop-in modules.
#   x_new = x + dropout(relu(LN(TransformerConv(x, graph, f))))
# with the edge features f (rows F[feat_row[t]] or F[t]) projected by M_h = W_e,h P (+ w̄ = W_e p).
# ------------------------------------------------------------------------------------------------
def proj_weights(We: torch.Tensor, Wp: torch.Tensor, bp: torch.Tensor):
    """M = W_edge @ W_proj and w̄ = W_edge @ b_proj, for one conv ([D,D]) or stacked layers
    ([L,D,D] strided views) in one batched GEMM each."""
    lead = We.shape[:-2]
    D = We.size(-1)
    M = torch.empty(*lead, D, D, device=We.device)
    wbar = torch.empty(*lead, D, device=We.device)
    ops.gemm(We, Wp, M)
    ops.gemm(We, bp.unsqueeze(-1), wbar.unsqueeze(-1))
    return M, wbar


def proj_grads(We, Wp, bp, dM, dwbar, gWe, gWp, gbp) -> None:
    """Chain rule through M = W_edge W_proj, w̄ = W_edge b_proj (batched over stacked layers):
    dW_edge = dM W_proj^T + dw̄ b_proj^T, dW_proj = W_edge^T dM, db_proj = W_edge^T dw̄."""
    ops.gemm(dM, Wp.transpose(-1, -2), gWe)
    ops.gemm(dwbar.unsqueeze(-1), bp.unsqueeze(-2), gWe, beta=1.0)
    ops.gemm(We.transpose(-1, -2), dM, gWp)
    ops.gemm(We.transpose(-1, -2), dwbar.unsqueeze(-1), gbp.unsqueeze(-1))


def proj_grads_shared(We, Wp, bp, dM, dwbar, gWe, gWp, gbp) -> None:
    """proj_grads for L stacked edge projections W_edge[l] that share ONE (W_proj, b_proj) — the
    angle encoder's second Linear folded into every line-graph conv: the shared gradients are the
    sums over layers (batch-reduced GEMMs)."""
    L = We.size(0)
    ops.gemm(dM, Wp.expand(L, *Wp.shape).transpose(-1, -2), gWe)
    ops.gemm(dwbar.unsqueeze(-1), bp.expand(L, bp.numel()).unsqueeze(-2), gWe, beta=1.0)
    ops.gemm(We.transpose(-1, -2), dM, gWp, reduce_batch=True)
    ops.gemm(We.transpose(-1, -2), dwbar.unsqueeze(-1), gbp.unsqueeze(-1), reduce_batch=True)


def block_forward(cv: _Conv, X: torch.Tensor, g: ops.GraphCSR, F: Optional[torch.Tensor], feat_row,
                  M: torch.Tensor, wbar: Optional[torch.Tensor], H: int, p_drop: float, seed_att: int,
                  seed_blk: int, side: Optional[torch.cuda.Stream] = None,
                  bf16_io: bool = False, X16: Optional[torch.Tensor] = None,
                  want_X16: bool = False, angle_x=None, Xa: Optional[torch.Tensor] = None, want_Xa: bool = False):
    """M: per-head edge projection [D, D] (W_edge, or W_edge W_proj); wbar: W_edge b_proj or None.
    bf16_io (bf16 storage, config C3 — the tensor dtypes of the reference's autocast, train.py:632-636):
    on a compacted graph the skip projection's output R and, in the backward, its gradient dR are
    bf16 (Linear outputs and their gradients); X16: a bf16 copy of X (the Linear's input as autocast
    casts it: bitwise the operand the bf16 matrix cores round X to) read by the skip projection and its
    weight gradient; want_X16: the gate kernel also writes a bf16 copy of the new state (c.Xn16).
    angle_x (the line graph, F None): (X, W1, b1, bf16) — the edge features are the angle encoder's
    hidden layer relu(X W1^T + b1), recomputed inside the attention kernels from the raw inputs X
    (ops.lg_fwd_x) instead of read; bf16: the bf16-storage form (K|V and f in bf16, config C3).
    On a compacted graph with a side stream the skip projection is queued there before the active-row
    gather and the Q/K/V product, so it overlaps those as well as the attention (+1 % at B = 32 against
    after them, rounds 3 and 5), and the gate reads the compacted conv output through the row map (no
    zero-filled [n, D] copy; the backward writes the compacted dout directly; +1.2 %, round 1).
    Xa: the active rows of X, already gathered (by the previous line block's gate kernel); want_Xa:
    this block's gate kernel writes the active rows of its new state to c.Xa_next.

    Compacted graphs (g.rows set: the graph's nodes are the active subset ``rows`` of X's rows, see
    BatchCache): Q/K/V, the attention and its per-node GEMMs run over the active rows only; the
    skip projection, gate, LayerNorm and residual over all rows (an inactive node's aggregated
    message is exactly 0: it has no in-edges)."""
    n, D = X.shape
    C = D // H
    dev = X.device
    c = _Ctx()
    c.X, c.F, c.feat_row = X, F, feat_row
    c.M, c.wbar = M, wbar
    c.rows = rows = g.rows
    with_proj = wbar is not None
    if rows is None:
        na = n
        QKVR = torch.empty(n, 4 * D, device=dev)
        ops.gemm(X, cv.Wqkvr.t(), QKVR, bias=cv.bqkvr)
        c.Xa, c.QKV, c.R = X, QKVR[:, :3 * D], QKVR[:, 3 * D:]
    else:
        na = g.n
        c.R = torch.empty(n, D, device=dev, dtype=torch.bfloat16 if bf16_io else torch.float32)
        Xs = X16 if (bf16_io and X16 is not None) else X   # the skip projection's A operand
        with _side_work(side, (X, Xs, c.R)):   # skip projection of all rows, beside Q/K/V and the attention
            ops.gemm(Xs, cv.Wqkvr[3 * D:].t(), c.R, bias=cv.bqkvr[3 * D:])
        c.Xa = Xa if Xa is not None else ops.gather_rows(X, rows)
        c.QKV = torch.empty(na, 3 * D, device=dev)
        ops.gemm(c.Xa, cv.Wqkvr[:3 * D].t(), c.QKV, bias=cv.bqkvr[:3 * D])
    c.X16 = X16 if (bf16_io and rows is not None) else None
    c.U = torch.empty(na, H, D, device=dev)
    ops.gemm(c.QKV[:, :D].view(na, H, C).transpose(0, 1), c.M.view(H, C, D), c.U.transpose(0, 1))
    c.outp_a = torch.empty(na, D, device=dev)
    c.S = torch.empty(na, H, D, device=dev)
    c.sumA = torch.empty(na, H, device=dev)
    c.mstat = torch.empty(na, H, device=dev)
    c.den = torch.empty(na, H, device=dev)
    c.KV16 = c.QKV16 = None
    c.angle_x = angle_x
    if angle_x is not None:
        Xa, W1, b1, bf = angle_x
        if bf:   # one bf16 copy of Q|K|V: K|V gathered by the attention, Q by the source-side backward
            c.QKV16 = ops.cast_bf16(c.QKV)
            c.KV16 = c.QKV16[:, D:3 * D]
        ops.lg_fwd_x(g, D, H, c.QKV, c.KV16, c.U, c.wbar, Xa, W1, b1, c.outp_a, c.S, c.sumA, c.mstat, c.den, p_drop,
                     seed_att)
    elif F is not None and F.dtype == torch.bfloat16 and feat_row is None:
        # bf16 storage (config C3), the line graph: the attention gathers K|V from a bf16 copy and streams
        # the bf16 angle hidden layer (the atom graph's bf16 bond-state rows go through tconv_fwd)
        # one bf16 copy of Q|K|V: K|V gathered by the attention, Q by the source-side backward
        c.QKV16 = ops.cast_bf16(c.QKV)
        c.KV16 = c.QKV16[:, D:3 * D]
        ops.lg_fwd_bf16(g, D, H, c.QKV, c.KV16, c.U, c.wbar, F, c.outp_a, c.S, c.sumA, c.mstat, c.den, p_drop, seed_att)
    else:
        ops.tconv_fwd(g, D, H, c.QKV, c.U, c.wbar, F, feat_row, c.outp_a, c.S, c.sumA, c.mstat, c.den, p_drop,
                      seed_att)
    if with_proj:
        ops.gemm(c.S.transpose(0, 1), c.M.view(H, C, D).transpose(1, 2), c.outp_a.view(na, H, C).transpose(0, 1),
                 beta=1.0, rowscale=c.sumA.t(), bias2=c.wbar.view(H, C))
    else:
        ops.gemm(c.S.transpose(0, 1), c.M.view(H, C, D).transpose(1, 2), c.outp_a.view(na, H, C).transpose(0, 1),
                 beta=1.0)
    c.outp_rows = None
    if rows is None:
        c.outp = c.outp_a
    else:
        c.outp, c.outp_rows = c.outp_a, g.cmap
    if side is not None and rows is not None:
        ops.stream_wait(torch.cuda.current_stream(dev), side)
    X_new = torch.empty(n, D, device=dev)
    c.Xn16 = torch.empty(n, D, device=dev, dtype=torch.bfloat16) if want_X16 else None
    c.beta = torch.empty(n, device=dev)
    c.mu = torch.empty(n, device=dev)
    c.rstd = torch.empty(n, device=dev)
    c.Xa_next = (torch.empty(na, D, device=dev) if (want_Xa and rows is not None and c.outp_rows is not None)
                 else None)
    ops.gate_ln_fwd(c.outp, c.R, cv.wbeta, X, cv.lnw, cv.lnb, X_new, c.beta, c.mu, c.rstd, p_drop, seed_blk,
                    outp_rows=c.outp_rows, Xnew16=c.Xn16, Xa_out=c.Xa_next)
    c.p, c.seed_att, c.seed_blk, c.H, c.with_proj = p_drop, seed_att, seed_blk, H, with_proj
    return X_new, c


def block_backward(cv: _Conv, gv: _Conv, c, g: ops.GraphCSR, dX: torch.Tensor, dF: Optional[torch.Tensor],
                   dF_accumulate: int, dM: Optional[torch.Tensor] = None,
                   dwbar: Optional[torch.Tensor] = None, side: Optional[torch.cuda.Stream] = None,
                   keep_edge_scalars: bool = False, gate_reduce_side: bool = False,
                   wgrad_early: int = 0, dX_add: Optional[torch.Tensor] = None,
                   dX_zero: bool = False) -> None:
    """dX: gradient w.r.t. the block output on entry, w.r.t. the block input on exit (in place).
    dF: gradient w.r.t. the edge-feature rows (written or accumulated at the rows the forward read).
    Parameter gradients go to gv (gate/LN grads with +=, the rest overwritten); with a projection
    (c.wbar set) the gradients of M and w̄ are written to dM / dwbar for :func:`proj_grads`.
    side: a second stream for the weight-gradient products (dM, dw̄, dW, db), which nothing
    downstream in the backward reads; they overlap the next block's latency-bound attention.  The
    caller joins the side stream before reading those gradients.
    keep_edge_scalars: leave (Vd, dz_e, alpha_e) on ``c.edge_scalars`` for the deferred angle-encoder
    backward (ops.enc_bwd; then dF is None).
    gate_reduce_side: the gate/LayerNorm parameter-gradient reduction on the side stream.
    wgrad_early: where the side stream's weight-gradient products are queued — 0: after the dX
    products; 1: once dQ is final, before the dX products; 2: those final after the target-side
    kernel (dM, dw̄, the skip projection's) right after it, the rest once dQ is final.
    dX_add: a second part of the incoming gradient (the atom block's edge-feature gradient), added
    to dX by the gate kernel (ops.gate_ln_bwd).  dX_zero: dX holds nothing yet (the last line
    block, whose output only the atom block beside it reads): the incoming gradient is dX_add."""
    n, D = c.X.shape
    H = c.H
    C = D // H
    dev = dX.device
    m = g.m
    rows = c.rows
    na = n if rows is None else g.n
    dout = torch.empty(n if c.outp_rows is None else na, D, device=dev)
    if rows is None:
        dQKVR = torch.empty(n, 4 * D, device=dev)
        dQKV, dR = dQKVR[:, :3 * D], dQKVR[:, 3 * D:]
    else:
        dQKV = torch.empty(na, 3 * D, device=dev)
        dR = torch.empty(n, D, device=dev, dtype=c.R.dtype)   # bf16 storage: the gradient of a bf16 output
    ops.gate_ln_bwd(dX, c.outp, c.R, cv.wbeta, cv.lnw, cv.lnb, c.beta, c.mu, c.rstd, dout, dR, gv.wbeta, gv.lnw,
                    gv.lnb, c.p, c.seed_blk, outp_rows=c.outp_rows, reduce_stream=side if gate_reduce_side else None,
                    dX_add=dX_add, dX_zero=dX_zero)
    Wb = cv.Wqkvr   # B operand [4D, D]
    dout_a = dout if (rows is None or c.outp_rows is not None) else ops.gather_rows(dout, rows)
    Vd = torch.empty(na, H, D, device=dev)
    ops.gemm(dout_a.view(na, H, C).transpose(0, 1), c.M.view(H, C, D), Vd.transpose(0, 1))
    Sz = torch.empty(na, H, D, device=dev)
    sigz = torch.empty(na, H, device=dev)
    dz_e = torch.empty(max(m, 1), H, device=dev)
    al_e = torch.empty(max(m, 1), H, device=dev)
    if c.angle_x is not None:
        if dF is not None:
            raise ValueError("recomputed edge features need the deferred angle-encoder backward (no dF)")
        Xa, W1, b1, _ = c.angle_x
        ops.lg_bwd_dst_x(g, D, H, c.QKV, c.KV16, c.U, Vd, c.wbar, Xa, W1, b1, dout_a, c.outp_a, c.mstat, c.den,
                         dQKV[:, :D], Sz, sigz, dz_e, al_e, c.p, c.seed_att)
    elif c.KV16 is not None:
        if dF is not None:
            raise ValueError("bf16 edge-feature storage needs the deferred angle-encoder backward (no dF)")
        ops.lg_bwd_dst_bf16(g, D, H, c.QKV, c.KV16, c.U, Vd, c.wbar, c.F, dout_a, c.outp_a, c.mstat, c.den, dQKV[:, :D], Sz, sigz,
                            dz_e, al_e, c.p, c.seed_att)
    else:
        ops.tconv_bwd_dst(g, D, H, c.QKV, c.U, Vd, c.wbar, c.F, c.feat_row, dout_a, c.outp_a, c.mstat, c.den,
                          dQKV[:, :D], Sz, sigz, dz_e, al_e, dF, dF_accumulate, c.p, c.seed_att)
    Qh = c.QKV[:, :D].view(na, H, C).permute(1, 2, 0)
    Oh = dout_a.view(na, H, C).permute(1, 2, 0)
    wg = (cv, gv, c, side, Qh, Oh, Sz, sigz, dout_a, dQKV, dR, dQKVR if rows is None else None, dM, dwbar, H, C, D)
    early = wgrad_early if side is not None else 0
    if early >= 2:
        _weight_grads(*wg, part="a")     # final once the target-side kernel is done
    if c.QKV16 is not None:
        # bf16 storage: the gathered target rows (Q, dout) from bf16 copies — half the traffic
        ops.tconv_bwd_src(g, D, H, c.QKV, dout_a, dz_e, al_e, dQKV[:, D:3 * D], Q16=c.QKV16[:, :D],
                          dout16=ops.cast_bf16(dout_a))
    else:
        ops.tconv_bwd_src(g, D, H, c.QKV, dout_a, dz_e, al_e, dQKV[:, D:3 * D])
    if keep_edge_scalars:
        c.edge_scalars = (Vd, dz_e, al_e)
    dQv = dQKV[:, :D].view(na, H, C).transpose(0, 1)
    Mt = c.M.view(H, C, D).transpose(1, 2)
    # critical path: dQ (+ its edge-projection terms), then dX
    if c.with_proj:
        ops.gemm(Sz.transpose(0, 1), Mt, dQv, beta=1.0, rowscale=sigz.t(), bias2=c.wbar.view(H, C))
    else:
        ops.gemm(Sz.transpose(0, 1), Mt, dQv, beta=1.0)
    if early:
        _weight_grads(*wg, part="b" if early >= 2 else "ab")
    if rows is None:
        ops.gemm(dQKVR, Wb, dX, beta=1.0)                               # residual + projections
    else:
        ops.gemm(dR, Wb[3 * D:], dX, beta=1.0)                          # residual + skip projection
        ops.gemm(dQKV, Wb[:3 * D], dX, beta=1.0, c_rows=rows)           # + Q/K/V projections (active rows)
    if not early:
        _weight_grads(*wg, part="ab")


def _weight_grads(cv, gv, c, side, Qh, Oh, Sz, sigz, dout_a, dQKV, dR, dQKVR, dM, dwbar, H, C, D,
                  part: str = "ab") -> None:
    """A conv block's weight-gradient products (dM, dw̄ or dW_edge, dW, db): off the critical path.
    part "a": those final after the target-side attention backward (dM / dw̄ / dW_edge and, on a
    compacted graph, the skip projection's dW, db); "b": the rest (the Q/K/V projections' dW, db,
    which read dQ and dK/dV)."""
    rows = c.rows
    with _side_work(side, (c.QKV, dout_a, Sz, sigz, c.S, c.sumA, dQKV, dR, c.X, c.X16, c.Xa)):
        if "a" in part:
            if c.with_proj:
                ops.gemm(Qh, Sz.transpose(0, 1), dM.view(H, C, D))
                ops.gemm(Oh, c.S.transpose(0, 1), dM.view(H, C, D), beta=1.0)
                # dw̄_h = Σ Q_h σz_h + dout_h ΣA_h in one weighted column-sum kernel
                ops.wcolsum2(c.QKV[:, :D], sigz, dout_a, c.sumA, dwbar)
            else:
                ops.gemm(Qh, Sz.transpose(0, 1), gv.We.view(H, C, D))           # dW_edge directly
                ops.gemm(Oh, c.S.transpose(0, 1), gv.We.view(H, C, D), beta=1.0)
            if rows is not None:
                ops.gemm(dR.t(), c.X if c.X16 is None else c.X16, gv.Wqkvr[3 * D:], rowsum=gv.bqkvr[3 * D:])
        if "b" in part:
            if rows is None:
                ops.gemm(dQKVR.t(), c.X, gv.Wqkvr, rowsum=gv.bqkvr)
            else:
                ops.gemm(dQKV.t(), c.Xa, gv.Wqkvr[:3 * D], rowsum=gv.bqkvr[:3 * D])


class _side_work:
    """Runs the enclosed launches on ``side`` after everything already queued on the current
    stream (no-op context without a side stream).  The tensors are marked as used by the side
    stream so the caching allocator does not hand their memory to the main stream early."""

    def __init__(self, side: Optional[torch.cuda.Stream], tensors, wait: bool = True):
        self.side, self.tensors, self.ctx, self.wait = side, tensors, None, wait

    def __enter__(self):
        if self.side is None:
            return self
        if self.wait:   # else the caller has ordered ``side`` after what the enclosed work reads
            ops.stream_wait(self.side, torch.cuda.current_stream(self.side.device))
        for t in self.tensors:
            if t is not None:
                t.record_stream(self.side)
        self.ctx = torch.cuda.stream(self.side)
        self.ctx.__enter__()
        return self

    def __exit__(self, *exc):
        if self.ctx is not None:
            self.ctx.__exit__(*exc)
        return False


# ------------------------------------------------------------------------------------------------
# Engine
# ------------------------------------------------------------------------------------------------
class AlignnEngine:
    """``mode``: 'hetero' -> [B, 2T] = [mean | logvar] (HeteroAlignnRegressor.forward),
    'base' -> [B, T] (AlignnRegressor.forward), 'embed' -> shared [B, D] (embed)."""

    WGRAD_SPLIT_MAX_T = 1_000_000
    ATOM_STREAM_MIN_T = 100_000

    def _atom_mode(self, T: int, E: int) -> int:
        if E <= 0:
            return 0
        return self.atom_stream if self.atom_stream >= 0 else (2 if T >= self.ATOM_STREAM_MIN_T else 0)

    def __init__(self, cfg: AlignnConfig):
        cfg.validate()
        self.cfg = cfg
        # workspaces, side/aux streams and device step seed of this engine's launches (ops.ExecContext)
        self.ctx = ops.ExecContext("engine")
        self.debug = None  # dict -> backward stores intermediate gradients (diagnostics only)
        # weight-gradient products on a second stream, overlapping the next block's attention
        self.overlap = True
        # forward: the line blocks' skip projection on the second stream beside the attention
        # (measured +1.2 % graphs/s on MI355X, profiles/r01/v7_sweep.log)
        self.overlap_forward = True
        # GEMM arithmetic: "fp32" (the reference's CPU path; exact fp32 MFMA) or "bf16" (bf16 MFMA
        # inputs, fp32 accumulation — the reference's CUDA autocast).  With
        # "bf16" (and bf16_storage) the line-graph attention also streams its largest operands as the
        # autocast Linear outputs they are — the angle hidden layer and the gathered K|V rows in bf16;
        # softmax, accumulation, LayerNorm and every other tensor stay fp32
        self.precision = "fp32"
        self.bf16_storage = True
        # the angle encoder's first Linear (11 inputs, T rows) and its weight/bias gradients as
        # streamed HBM-rate kernels (skinny.hip) instead of MFMA tiles (+3.2 %, v7_sweep.log)
        self.skinny_encoder = True
        # angle encoder backward deferred to one pass after the last line block (ops.enc_bwd): the
        # line convs leave per-edge scalars instead of read-modify-writing a [T, D] gradient per layer
        # (+4.0 % graphs/s on MI355X once enc_bwd was column-parallel, profiles/r01/v13_sweep.log)
        self.defer_angle_bwd = True
        # gate/LayerNorm parameter-gradient reduction on the side stream (off the critical path)
        # (round 1: +0.3 %, v34_sweep_gate_reduce_side.log).  Round 5 re-sweep on the main stream: C3 +1.9 %
        # (23,292-23,363 -> 23,712-23,823 graphs/s), C2 +1.5 % beside the settings below (10,091-10,104
        # -> 10,247-10,255; profiles/r05/v15_sweep_engine_*.txt)
        self.gate_reduce_side = False
        # deferred angle-encoder backward on a third stream (see _backward): 1 always, 0 never, or
        # from this many line-graph edges on.  B = 32 (253,440 triplets): -0.6 %
        # (v31_sweep_enc_bwd_aux_rejected.log); B = 256 bf16 (2.03 M triplets, enc_bwd 1.06 ms, the
        # step's last branch): +1.8 % (17,697-17,740 -> 18,027-18,051 graphs/s,
        # profiles/r02/v30_ab_enc_bwd_aux_c3.log).  Round 5 (atom blocks on the aux stream at B = 32
        # too): B = 32 +1.1 % (9,972-9,985 -> 10,077-10,090 graphs/s), B = 256 bf16 within noise:
        # always (profiles/r05/v15_sweep_engine_c2.txt)
        self.enc_bwd_aux = 1
        # backward: where each block's weight-gradient products are queued on the side stream (see
        # block_backward: 0 after its dX products, 1 before them, 2 split at the target-side kernel);
        # -1: 2 below WGRAD_SPLIT_MAX_T line-graph edges, else 1.  B = 32: 0 -> 2 +2.3 % (8,842 ->
        # 9,043 graphs/s); B = 256 bf16: 2 measured -0.7 %, 1 +0.3 % (v20_ab_wgrad_levels.log)
        self.wgrad_early = -1
        # atom-graph blocks (NodeUpdateBlock) beside the line-graph blocks they do not depend on
        # (forward: atom block l || line block l+1; backward: atom block l-1 || line block l).  0:
        # inline, their edge-feature gradient accumulated into the bond-state gradient by the
        # attention kernel; 1: inline, that gradient into a buffer of its own, added by the next line
        # block's gate kernel (ops.gate_ln_bwd dX_add); 2: as 1 with the atom blocks on the aux stream
        # (bitwise equal to 1); -1: 2 from ATOM_STREAM_MIN_T line-graph edges on, else 0.  B = 256
        # bf16: 0 -> 2 +2.6 % (18,963 -> 19,458 graphs/s); B = 32: 2 within noise of 0 (-0.5 %),
        # 1 -0.6 % (profiles/r03/v21_ab_atom_stream.log).  Round 5, with the faster line-graph and
        # GEMM kernels, B = 32 (253,440 line-graph edges): 0 -> 2 +2.9 % (9,652-9,670 -> 9,929-9,957
        # graphs/s; 1 -0.8 %, profiles/r05/v15_sweep_engine_c2.txt): ATOM_STREAM_MIN_T 1 M -> 100,000
        self.atom_stream = -1
        # bf16 storage: the atom blocks' edge-feature gradient (the gradient autocast returns through
        # its bf16 cast of the bond states) stored in bf16 between the atom attention backward that
        # writes it and the line block's gate kernel that adds it (half the bytes of both)
        self.bf16_atom_grad = True
        # with the atom blocks on the aux stream: the node encoder and the atom projection folds there
        # too (forward prologue)
        self.encoders_aux = True
        # each line block's gate kernel also writes the active rows of the new bond state, which the
        # next line block reads instead of gathering them in a launch of its own
        self.gate_gathers = True
        # the line convs' edge features (the angle encoder's hidden layer, [T, 256]) recomputed inside
        # the attention kernels from the 11 raw inputs instead of materialised and re-read 8 times
        # (ops.lg_fwd_x / lg_bwd_dst_x; the deferred encoder backward recomputes its ReLU mask)
        self.recompute_angle = True
        # ... and at bf16 storage (config C3): opt-in — the matrix-core attention kernels (lgmx.hip)
        # recompute it as autocast does and take every per-edge product on the matrix cores.  Off by
        # default: C3 21.8k vs 23.2k graphs/s against the streamed bf16 rows on the same box
        # (profiles/r06/ab_c3_recompute_mx.txt; the per-target kernels are issue- and latency-bound at
        # 0.13 of the matrix cores).  Off, the stored layer is autocast's Linear on the matrix cores
        # (ops.linear_smallk_bf16) and the deferred encoder backward recomputes its mask from x.
        self.recompute_angle_bf16 = False

    @contextmanager
    def using_precision(self, precision: str):
        """Runs the enclosed calls at ``precision`` ("fp32" / "bf16"), then restores the engine's own
        (the module API's per-call autocast precision, model._autocast_dtype)."""
        if precision not in ("fp32", "bf16"):
            raise ValueError(f"precision must be 'fp32' or 'bf16', got {precision!r}")
        prev, self.precision = self.precision, precision
        try:
            yield
        finally:
            self.precision = prev

    def _bf16_io(self, D: int) -> bool:
        """bf16 storage of the line blocks' skip projection (R, dR) and of the bond state's bf16 copy
        (precision "bf16" with bf16_storage: autocast's dtypes, train.py:632-636)."""
        return self.precision == "bf16" and self.bf16_storage and D % 4 == 0

    def _bf16_angle(self, bc, D: int) -> bool:
        """bf16 storage of the angle hidden layer and the line graph's K|V rows: precision "bf16", the
        deferred encoder backward, and a line graph in the bf16 kernels' domain (D = 256, H <= 4,
        single-wave work items without heavy nodes)."""
        if not (self.precision == "bf16" and self.bf16_storage and self.defer_angle_bwd and D == 256
                and self.cfg.heads in (1, 2, 4) and bc.lg is not None and bc.lg.policy.wave_items
                and ops.enc_bwd_ok(D, self.cfg.heads, self.cfg.layers, bc.xa.size(1))):
            return False
        return bc.lg.schedule().n_heavy == 0

    def _angle_xf(self, bc, D: int) -> bool:
        """The line convs recompute their edge features (recompute_angle): D = 256, H = 4, 11 raw
        angle inputs, the deferred encoder backward, a single-wave-item line-graph schedule.  fp32: only
        where the materialised layer would come from linear_smallk (skinny_encoder), whose fma chain the
        recompute reproduces bit for bit."""
        if self.precision == "bf16" and self.bf16_storage and not self.recompute_angle_bf16:
            return False
        if not (self.precision == "bf16" and self.bf16_storage) and not self.skinny_encoder:
            return False
        return bool(self.recompute_angle and self.defer_angle_bwd and bc.xa is not None and bc.lg is not None
                    and ops.lg_x_ok(bc.lg, D, self.cfg.heads, bc.xa)
                    and ops.enc_bwd_ok(D, self.cfg.heads, self.cfg.layers, bc.xa.size(1)))

    def _angle_hidden(self, P: FlatViews, bc: BatchCache, D: int, dev, a: torch.Tensor) -> None:
        """a = relu(x_angle W1^T + b1), the angle encoder's hidden layer (its 2nd Linear is folded).
        bf16 ``a``: config C3 (autocast) — a bf16 Linear output, read by the bf16-storage line-graph
        attention (its backward is the deferred enc_bwd)."""
        W1, b1 = P.enc("angle", 0, "weight"), P.enc("angle", 0, "bias")
        if a.dtype == torch.bfloat16:
            if self._angle_mx(bc, W1, a):
                ops.linear_smallk_bf16(bc.xa, W1, b1, a, relu=True)
            else:
                a32 = torch.empty(a.shape, device=dev)
                ops.gemm(bc.xa, W1.t(), a32, bias=b1, relu=True)
                ops.cast_bf16(a32, a)
        elif self.skinny_encoder and ops.linear_smallk_ok(bc.xa, W1, a):
            ops.linear_smallk(bc.xa, W1, b1, a, relu=True)
        else:
            ops.gemm(bc.xa, W1.t(), a, bias=b1, relu=True)

    def _angle_mx(self, bc: BatchCache, W1: torch.Tensor, a: Optional[torch.Tensor]) -> bool:
        """The bf16 hidden layer is autocast's Linear on the matrix cores (ops.linear_smallk_bf16): its
        ReLU mask is then the one the deferred encoder backward recomputes from x, bit for bit."""
        return (a is not None and a.dtype == torch.bfloat16 and self.skinny_encoder
                and ops.linear_smallk_bf16_ok(bc.xa, W1, a))

    def _line_proj(self, P: FlatViews, ctx, L: int, D: int) -> None:
        """The line convs' edge projections with the angle encoder's second Linear folded in."""
        W2, b2 = P.enc("angle", 2, "weight"), P.enc("angle", 2, "bias")
        ctx.Ml_all, ctx.wl_all = proj_weights(P.edge_We, W2.expand(L, D, D), b2.expand(L, D))

    def _mlp_fwd(self, x, W1, b1, W2, b2):
        D = self.cfg.hidden
        h1 = torch.empty(x.size(0), D, device=x.device)
        ops.gemm(x, W1.t(), h1, bias=b1, relu=True)
        out = torch.empty(x.size(0), D, device=x.device)
        ops.gemm(h1, W2.t(), out, bias=b2)
        return h1, out

    def _mlp_bwd(self, dout, x, h1, W2, gW1, gb1, gW2, gb2):
        ops.gemm(dout.t(), h1, gW2, rowsum=gb2)   # the bias gradient from the same launch
        dh1 = torch.empty_like(h1)
        ops.gemm(dout, W2, dh1, mask=h1)
        ops.gemm(dh1.t(), x, gW1, rowsum=gb1)

    def forward(self, P: FlatViews, batch, bc: BatchCache, training: bool, seed: int = 0,
                x: Optional[torch.Tensor] = None, global_x: Optional[torch.Tensor] = None, mode: str = "hetero"):
        with ops.using(self.ctx), ops.gemm_precision(self.precision):
            return self._forward(P, batch, bc, training, seed, x, global_x, mode)

    def backward(self, P: FlatViews, G: FlatViews, ctx, dout: torch.Tensor, between=None) -> None:
        """Writes d(loss)/d(param) for every parameter into G: the per-layer backward, then
        ``between()`` (if given), then the tail.  When ``between`` runs, the gradients of the conv
        blocks' own parameters (flat [0, layout.bucket_split)) are final on the main and side streams
        — the first data-parallel bucket (dp.GradBuckets) can be reduced while the tail runs."""
        t = self.backward_layers(P, G, ctx, dout)
        if between is not None:
            between()
        self.backward_tail(t)

    def backward_layers(self, P: FlatViews, G: FlatViews, ctx, dout: torch.Tensor):
        """Heads, readout and the L x (node block, edge block) backward; returns the tail's state."""
        with ops.using(self.ctx), ops.gemm_precision(self.precision):
            self.ctx.new_pass()
            return self._backward_layers(P, G, ctx, dout)

    def backward_tail(self, t) -> None:
        """The edge-projection chain rules, the deferred angle-encoder backward and the encoder MLPs'
        backward, then the join of every stream into the current one."""
        with ops.using(self.ctx), ops.gemm_precision(self.precision):
            self._backward_tail(t)

    def _forward(self, P: FlatViews, batch, bc: BatchCache, training: bool, seed: int = 0,
                 x: Optional[torch.Tensor] = None, global_x: Optional[torch.Tensor] = None, mode: str = "hetero"):
        cfg = self.cfg
        D, H, L = cfg.hidden, cfg.heads, cfg.layers
        p_drop = cfg.dropout if training else 0.0
        dev = batch.x.device
        N, E, T, B = bc.N, bc.E, bc.T, bc.B
        ctx = _Ctx()
        ctx.seed, ctx.p, ctx.mode = seed, p_drop, mode
        x = (batch.x if x is None else x).contiguous()
        global_x = (batch.global_x if global_x is None else global_x).contiguous()
        ctx.x = x
        edge_attr = batch.edge_attr.contiguous()
        ctx.edge_attr = edge_attr
        # Angle encoder (train.py:553-554): only its hidden layer is materialised.  Its second Linear
        # (W2, b2) is folded into every line-graph conv's edge projection, M_l = W_edge,l W2 and
        # w̄_l = W_edge,l b2 — exact algebra, so the [T, D] x [D, D] GEMM and its two
        # backward GEMMs never run.
        ctx.has_angle = cfg.angle_dim > 0 and bc.xa is not None
        side = ops.side_stream(dev) if (self.overlap and self.overlap_forward) else None
        # the line convs recompute the angle hidden layer from the raw inputs (no [T, D] array)
        xf = ctx.has_angle and T > 0 and E > 0 and L > 0 and self._angle_xf(bc, D)
        angle_x = None
        if xf:
            angle_x = (bc.xa, P.enc("angle", 0, "weight"), P.enc("angle", 0, "bias"), self._bf16_angle(bc, D))
        ctx.angle_x = angle_x
        # the angle encoder's first Linear on the side stream beside the node/edge encoders (round 3)
        angle_side = side is not None and ctx.has_angle and not xf
        if xf:
            a = None
        elif ctx.has_angle:
            a = torch.empty(T, D, device=dev, dtype=torch.bfloat16 if self._bf16_angle(bc, D) else torch.float32)
        else:
            a = ops.zeros(T, D, device=dev)
        if angle_side:
            # beside the node/edge encoders; the main stream waits for it before the first line block
            with _side_work(side, (a,)):
                self._angle_hidden(P, bc, D, dev, a)
        line_proj = T > 0 and E > 0 and L > 0 and ctx.has_angle
        # atom blocks on the aux stream: atom block l waits for line block l, line block l+1 does not
        # wait for it (it reads only the bond states); the readout joins the aux stream
        aux = ops.aux_stream(dev) if (self._atom_mode(T, E) == 2 and side is not None) else None
        # encoders (train.py:547-556).  With the atom blocks on the aux stream, the node encoder and the
        # atom blocks' projection folds (what only atom block 0 reads) run there too, beside the edge
        # encoder and the first line block
        atom_pre = aux is not None and self.encoders_aux
        if atom_pre:
            with _side_work(aux, (x,)):
                ctx.h1n, h = self._mlp_fwd(x, P.enc("node", 0, "weight"), P.enc("node", 0, "bias"),
                                           P.enc("node", 2, "weight"), P.enc("node", 2, "bias"))
                if E > 0 and L > 0:
                    ctx.M_all, ctx.wbar_all = proj_weights(P.node_We, P.node_Wp, P.node_bp)
        else:
            ctx.h1n, h = self._mlp_fwd(x, P.enc("node", 0, "weight"), P.enc("node", 0, "bias"),
                                       P.enc("node", 2, "weight"), P.enc("node", 2, "bias"))
        if edge_attr.numel() > 0:
            ctx.h1e, e = self._mlp_fwd(edge_attr, P.enc("edge", 0, "weight"), P.enc("edge", 0, "bias"),
                                       P.enc("edge", 2, "weight"), P.enc("edge", 2, "bias"))
        else:
            ctx.h1e, e = None, ops.zeros(E, D, device=dev)
        if angle_side:
            ops.stream_wait(torch.cuda.current_stream(dev), side)
        elif ctx.has_angle and not xf:
            self._angle_hidden(P, bc, D, dev, a)
        ctx.h1a = ctx.a = a
        ctx.a_mx = ctx.has_angle and self._angle_mx(bc, P.enc("angle", 0, "weight"), a)
        ctx.edge, ctx.node = [], []
        if line_proj:
            self._line_proj(P, ctx, L, D)
        if E > 0 and L > 0 and not atom_pre:
            ctx.M_all, ctx.wbar_all = proj_weights(P.node_We, P.node_Wp, P.node_bp)
        bf16_io = self._bf16_io(D) and bc.lg is not None and bc.lg.rows is not None
        e16 = None   # bf16 copy of the bond state (written by the previous line block's gate kernel)
        ea = None    # its active rows (likewise)
        for l in range(L):
            # EdgeUpdateBlock (train.py:312-317): line graph, angle embedding in target-sorted order
            if T > 0 and E > 0:
                Ml, wl = (ctx.Ml_all[l], ctx.wl_all[l]) if ctx.has_angle else (P.edge[l].We, None)
                e, c = block_forward(P.edge[l], e, bc.lg, a, None, Ml, wl, H, p_drop,
                                     site_seed(seed, 4 * l), site_seed(seed, 4 * l + 1), side=side,
                                     bf16_io=bf16_io, X16=e16, want_X16=bf16_io, angle_x=angle_x,
                                     Xa=ea, want_Xa=self.gate_gathers and l + 1 < L)
                e16 = c.Xn16
                ea = c.Xa_next
            else:
                c = None
            ctx.edge.append(c)
            # NodeUpdateBlock (train.py:330-336): atom graph, bond states gathered through the CSR perm
            if E > 0:
                # bf16 storage: the bond-state rows as autocast hands them to edge_proj (bf16: the gate
                # kernel's copy), and the line graph's source-side backward gathers Q / dout as bf16 copies
                ef = e16 if (bf16_io and e16 is not None) else e
                with _side_work(aux, (e, ef, h, ctx.M_all, ctx.wbar_all)):
                    h, c = block_forward(P.node[l], h, bc.ag, ef, bc.ag.perm_dst, ctx.M_all[l], ctx.wbar_all[l], H,
                                         p_drop, site_seed(seed, 4 * l + 2), site_seed(seed, 4 * l + 3))
            else:
                c = None
            ctx.node.append(c)
        if aux is not None:
            ops.stream_wait(torch.cuda.current_stream(dev), aux)
        ctx.h = h
        # readout (train.py:562-574)
        gdim = global_x.numel() // max(B, 1)
        sg = batch.sg_one_hot.contiguous()
        sgdim = sg.numel() // max(B, 1)
        if gdim + sgdim != cfg.global_dim:
            raise ValueError(f"global features: got {gdim}+{sgdim}, model expects {cfg.global_dim}")
        W = D + gdim + sgdim
        ctx.feats = torch.empty(B, W, device=dev)
        ops.readout_feats_fwd(h, bc.ptr, global_x, gdim, sg, sgdim, ctx.feats, p_drop, site_seed(seed, 4 * L))
        ctx.pre = torch.empty(B, D, device=dev)
        ops.gemm(ctx.feats, P.named[P.prefix + "feat_proj.0.weight"].t(), ctx.pre,
                 bias=P.named[P.prefix + "feat_proj.0.bias"], relu=True)
        ctx.shared = torch.empty(B, D, device=dev)
        ops.dropout(ctx.pre, ctx.shared, None, p_drop, site_seed(seed, 4 * L + 1))
        ctx.bc = bc
        Tt = cfg.target_dim
        if mode == "embed":
            return ctx.shared, ctx
        if mode == "hetero":
            out = torch.empty(B, 2 * Tt, device=dev)
            dw = P.Wlogvar.storage_offset() - P.Wmean.storage_offset()
            db = P.blogvar.storage_offset() - P.bmean.storage_offset()
            if (dw > 0 and db > 0 and P.Wmean.is_contiguous() and P.Wlogvar.is_contiguous()
                    and P.Wmean.untyped_storage().data_ptr() == P.Wlogvar.untyped_storage().data_ptr()
                    and P.bmean.untyped_storage().data_ptr() == P.blogvar.untyped_storage().data_ptr()):
                # both heads in one batched launch (the flat parameter buffer holds them at a fixed
                # distance): the same per-head products as two launches, bit for bit
                Wb = torch.as_strided(P.Wmean, (2, D, Tt), (dw, 1, D))
                bb = torch.as_strided(P.bmean, (2, Tt), (db, 1))
                ops.gemm(ctx.shared, Wb, torch.as_strided(out, (2, B, Tt), (Tt, 2 * Tt, 1)), bias=bb)
            else:
                ops.gemm(ctx.shared, P.Wmean.t(), out[:, :Tt], bias=P.bmean)
                ops.gemm(ctx.shared, P.Wlogvar.t(), out[:, Tt:], bias=P.blogvar)
            return out, ctx
        out = torch.empty(B, Tt, device=dev)
        ops.gemm(ctx.shared, P.Wout.t(), out, bias=P.bout)
        return out, ctx

    def _backward_layers(self, P: FlatViews, G: FlatViews, ctx, dout: torch.Tensor):
        """Writes d(loss)/d(param) for every parameter into G (overwrites; head grads are zero in
        'embed' mode) together with _backward_tail.  ``dout`` is the gradient of the forward's output."""
        cfg = self.cfg
        D, L = cfg.hidden, cfg.layers
        Tt = cfg.target_dim
        bc = ctx.bc
        N, E, T, B = bc.N, bc.E, bc.T, bc.B
        dev = dout.device
        p_drop, seed = ctx.p, ctx.seed
        pre = P.prefix
        g = G.named
        ops.zero_(G.flat)
        dout = dout.contiguous()
        side = ops.side_stream(dev) if self.overlap else None
        # heads (train.py:582-585); their weight gradients on the side stream (off the dh chain)
        if ctx.mode == "embed":
            dshared = dout
        else:
            dshared = torch.empty(B, D, device=dev)
            if ctx.mode == "hetero":
                with _side_work(side, (dout, ctx.shared)):
                    ops.gemm(dout[:, :Tt].t(), ctx.shared, G.Wmean, rowsum=G.bmean)
                    ops.gemm(dout[:, Tt:].t(), ctx.shared, G.Wlogvar, rowsum=G.blogvar)
                ops.gemm(dout[:, :Tt], P.Wmean, dshared)
                ops.gemm(dout[:, Tt:], P.Wlogvar, dshared, beta=1.0)
            else:
                with _side_work(side, (dout, ctx.shared)):
                    ops.gemm(dout.t(), ctx.shared, G.Wout, rowsum=G.bout)
                ops.gemm(dout, P.Wout, dshared)
        # feat_proj + readout (train.py:562-573)
        dpre = torch.empty(B, D, device=dev)
        ops.dropout(dshared, dpre, ctx.pre, p_drop, site_seed(seed, 4 * L + 1))
        Wf = P.named[pre + "feat_proj.0.weight"]
        with _side_work(side, (dpre, ctx.feats)):
            ops.gemm(dpre.t(), ctx.feats, g[pre + "feat_proj.0.weight"], rowsum=g[pre + "feat_proj.0.bias"])
        Wfeat = ctx.feats.size(1)
        dfeats = torch.empty(B, Wfeat, device=dev)   # the pooling backward reads its first D columns only
        ops.gemm(dpre, Wf[:, :D], dfeats[:, :D])
        dh = torch.empty(N, D, device=dev)
        ops.readout_pool_bwd(dfeats, bc.ptr, bc.batch_vec, dh, False, p_drop, site_seed(seed, 4 * L))
        atom_mode = self._atom_mode(T, E)
        # the last line block's output feeds only the atom block beside it, whose edge-feature gradient
        # (dF_atom, atom_mode >= 1) is that block's whole incoming gradient: its gate kernel writes de
        # from it instead of adding it to a zero-filled de (ops.gate_ln_bwd dX_zero)
        de_fresh = (atom_mode >= 1 and L > 0 and T > 0 and self.debug is None and ctx.edge[L - 1] is not None
                    and ctx.node[L - 1] is not None)
        de = torch.empty(E, D, device=dev) if de_fresh else ops.zeros(E, D, device=dev)
        defer = (self.defer_angle_bwd and ctx.has_angle and T > 0 and E > 0 and L > 0
                 and ops.enc_bwd_ok(D, cfg.heads, L, bc.xa.size(1)))
        da = torch.empty(T, D, device=dev) if (T > 0 and not defer) else None
        da_written = False
        if E > 0 and L > 0:
            dM_all = torch.empty(L, D, D, device=dev)
            dwbar_all = torch.empty(L, D, device=dev)
        line_proj = T > 0 and E > 0 and L > 0 and ctx.has_angle
        wgrad = self.wgrad_early if self.wgrad_early >= 0 else (2 if T < self.WGRAD_SPLIT_MAX_T else 1)
        if line_proj:
            dMl_all = torch.empty(L, D, D, device=dev)
            dwl_all = torch.empty(L, D, device=dev)
        # atom_stream 1/2: each atom block's edge-feature gradient into a buffer of its own, added to
        # the bond-state gradient before the line block's backward; 2: the atom blocks on the aux
        # stream, atom block l-1 beside line block l (it reads only dh and its own forward state)
        # bf16 storage: the atom blocks' edge-feature gradient as autocast returns it through the bf16
        # cast of the bond states for edge_proj (train.py:325/:333 under :632-636) — written by the atom
        # attention backward, read by the next line block's gate kernel
        df_bf16 = self.bf16_atom_grad and self._bf16_io(D) and T > 0 and self.debug is None
        dF_atom = (torch.empty(L, E, D, device=dev, dtype=torch.bfloat16 if df_bf16 else torch.float32)
                   if atom_mode else None)
        aux = ops.aux_stream(dev) if (atom_mode == 2 and side is not None) else None

        def atom_bwd(l):
            c = ctx.node[l]
            if c is None:
                return
            if atom_mode:
                block_backward(P.node[l], G.node[l], c, bc.ag, dh, dF_atom[l], 0, dM_all[l], dwbar_all[l],
                               side=side, gate_reduce_side=self.gate_reduce_side, wgrad_early=wgrad)
            else:
                block_backward(P.node[l], G.node[l], c, bc.ag, dh, de, True, dM_all[l], dwbar_all[l], side=side,
                               gate_reduce_side=self.gate_reduce_side, wgrad_early=wgrad)

        if aux is not None and L > 0:
            with _side_work(aux, (dh, dF_atom, dM_all, dwbar_all)):
                atom_bwd(L - 1)
        for l in reversed(range(L)):
            if self.debug is not None:
                self.debug[f"dh{l + 1}"], self.debug[f"de{l + 1}_pre"] = dh.clone(), de.clone()
            if aux is None:
                atom_bwd(l)
            else:
                ops.stream_wait(torch.cuda.current_stream(dev), aux)   # atom block l is done
                if l > 0:
                    with _side_work(aux, (), wait=False):   # ordered after atom block l on aux
                        atom_bwd(l - 1)
            add = dF_atom[l] if (atom_mode and ctx.node[l] is not None) else None
            if add is not None and (ctx.edge[l] is None or self.debug is not None):
                ops.add_(de, add)   # no line block to fold it into (or debug wants de complete here)
                add = None
            if self.debug is not None:
                self.debug[f"de{l + 1}"] = de.clone()
            c = ctx.edge[l]
            if c is not None:
                # dF of the line convs is the gradient of the angle hidden layer, summed over layers;
                # the last (l = 0) applies the ReLU mask in place
                flags = (1 if da_written else 0) | (2 if (ctx.has_angle and l == 0) else 0)
                if line_proj:
                    block_backward(P.edge[l], G.edge[l], c, bc.lg, de, da, flags, dMl_all[l], dwl_all[l], side=side,
                                   keep_edge_scalars=defer, gate_reduce_side=self.gate_reduce_side,
                                   wgrad_early=wgrad, dX_add=add, dX_zero=de_fresh and l == L - 1)
                else:
                    block_backward(P.edge[l], G.edge[l], c, bc.lg, de, da, flags, side=side,
                                   gate_reduce_side=self.gate_reduce_side,
                                   wgrad_early=wgrad, dX_add=add, dX_zero=de_fresh and l == L - 1)
                da_written = True
        t = _Ctx()
        t.P, t.G, t.ctx, t.bc, t.dh, t.de, t.da, t.defer, t.side, t.line_proj = P, G, ctx, bc, dh, de, da, defer, side, line_proj
        t.da_written = da_written
        if E > 0 and L > 0:
            t.dM_all, t.dwbar_all = dM_all, dwbar_all
        if line_proj:
            t.dMl_all, t.dwl_all = dMl_all, dwl_all
        return t

    def _backward_tail(self, t) -> None:
        cfg = self.cfg
        L = cfg.layers
        P, G, ctx, bc, dh, de, da, defer, side, line_proj = (t.P, t.G, t.ctx, t.bc, t.dh, t.de, t.da, t.defer, t.side,
                                                             t.line_proj)
        da_written = t.da_written
        N, E, T = bc.N, bc.E, bc.T
        dev = dh.device
        if E > 0 and L > 0:
            dM_all, dwbar_all = t.dM_all, t.dwbar_all
        if line_proj:
            dMl_all, dwl_all = t.dMl_all, t.dwl_all
        if self.debug is not None:
            self.debug["de0"] = de.clone()
        # projection chain rules and the angle encoder's first layer: side stream (after the
        # per-layer dM/dw̄ there), overlapping the edge/node encoder backward below
        kept = [t for c in ctx.edge for t in (c.U, *c.edge_scalars)] if defer else []
        # bf16 storage: the deferred backward on the matrix cores in bf16, its ReLU mask read from the
        # forward's bf16 hidden layer (alignn_enc_bwd_bf16; C3 +3.7 %, profiles/r03/v14_*).  fp32 keeps
        # the VALU kernel: exact fp32 MFMA runs at the VALU rate and measured slower (v15_*)
        f_rows = (ctx.a if (defer and ctx.a is not None and ctx.a.dtype == torch.bfloat16 and ctx.a.dim() == 2
                            and ctx.a.size(1) == 256 and cfg.heads % 2 == 0) else None)
        # recomputed edge features: the bf16 form recomputes its ReLU mask from the raw inputs too
        enc16 = defer and ctx.angle_x is not None and ctx.angle_x[3]
        if f_rows is not None:
            kept.append(f_rows)
            # a stored layer from the matrix-core Linear: the mask recomputed from the 11 raw inputs is the
            # stored one's bit for bit, and cheaper than reading the [T, 256] rows back (enc_bwd_bf16_x)
            if getattr(ctx, "a_mx", False) and bc.xa.size(1) <= ops.ENC_XF_KMAX:
                f_rows, enc16 = None, True
        # the deferred angle-encoder backward (the longest branch of the tail) on a third stream,
        # started as soon as the last line block is done instead of behind the side stream's queue
        use_aux = self.enc_bwd_aux == 1 or (self.enc_bwd_aux > 1 and T >= self.enc_bwd_aux)
        aux = ops.aux_stream(dev) if (defer and side is not None and use_aux) else None
        if aux is not None:
            with _side_work(aux, kept):
                ops.enc_bwd(bc.lg, bc.xa, P.enc("angle", 0, "weight"), P.enc("angle", 0, "bias"),
                            [c.U for c in ctx.edge], [c.edge_scalars[0] for c in ctx.edge],
                            [c.edge_scalars[1] for c in ctx.edge], [c.edge_scalars[2] for c in ctx.edge],
                            G.enc("angle", 0, "weight"), G.enc("angle", 0, "bias"), F=f_rows, bf16=enc16)
        with _side_work(side, (da, *kept)):
            if E > 0 and L > 0:
                proj_grads(P.node_We, P.node_Wp, P.node_bp, dM_all, dwbar_all, G.node_We, G.node_Wp, G.node_bp)
            if line_proj:
                proj_grads_shared(P.edge_We, P.enc("angle", 2, "weight"), P.enc("angle", 2, "bias"), dMl_all,
                                  dwl_all, G.edge_We, G.enc("angle", 2, "weight"), G.enc("angle", 2, "bias"))
            if defer:
                if aux is None:
                    ops.enc_bwd(bc.lg, bc.xa, P.enc("angle", 0, "weight"), P.enc("angle", 0, "bias"),
                                [c.U for c in ctx.edge], [c.edge_scalars[0] for c in ctx.edge],
                                [c.edge_scalars[1] for c in ctx.edge], [c.edge_scalars[2] for c in ctx.edge],
                                G.enc("angle", 0, "weight"), G.enc("angle", 0, "bias"), F=f_rows, bf16=enc16)
            elif ctx.has_angle and da_written:
                # da is the masked hidden-layer gradient
                if self.skinny_encoder and bc.xa.size(1) <= ops.SMALLN_MAX:
                    ops.gemm_tn_smalln(da, bc.xa, G.enc("angle", 0, "weight"), colsum=G.enc("angle", 0, "bias"))
                else:
                    ops.gemm(da.t(), bc.xa, G.enc("angle", 0, "weight"))
                    ops.colsum(da, G.enc("angle", 0, "bias"))
        if ctx.h1e is not None:
            self._mlp_bwd(de, ctx.edge_attr, ctx.h1e, P.enc("edge", 2, "weight"), G.enc("edge", 0, "weight"),
                          G.enc("edge", 0, "bias"), G.enc("edge", 2, "weight"), G.enc("edge", 2, "bias"))
        self._mlp_bwd(dh, ctx.x, ctx.h1n, P.enc("node", 2, "weight"), G.enc("node", 0, "weight"),
                      G.enc("node", 0, "bias"), G.enc("node", 2, "weight"), G.enc("node", 2, "bias"))
        if side is not None:
            ops.stream_wait(torch.cuda.current_stream(dev), side)  # join: every gradient is written
        if aux is not None:
            ops.stream_wait(torch.cuda.current_stream(dev), aux)
